"""Eager bs32 bf16 eval forward of PoseNetRGBDGeometric between two marker launches
(pose6d_pinhole_z_fwd, never launched by this model), for rocprofv3 --pmc passes:
every kernel of `--reps` forwards is a dispatch of its own, in forward order.
tools/eval_pmc_summary.py joins the passes per launch position.
    rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d OUT -o run --output-format csv -- python3 tools/eval_pmc.py"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "6d-pose-estimation_amd")]

import torch  # noqa: E402

from bench import synth_batch  # noqa: E402
from tools.step_profile import marker  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    from models.pose_net_rgbd_geometric import PoseNetRGBDGeometric
    dev = torch.device("cuda")
    torch.manual_seed(0)
    m = PoseNetRGBDGeometric(pretrained=False).to(dev).set_compute_dtype(torch.bfloat16).eval()
    b = synth_batch(32, dev, seed=1)
    args = (b[0], None, b[1], b[2], b[3])
    with torch.no_grad():
        for _ in range(3):
            m(*args)
        torch.cuda.synchronize()
        marker()
        for _ in range(a.reps):
            m(*args)
        marker()
    torch.cuda.synchronize()
    print("reps", a.reps)


if __name__ == "__main__":
    main()
