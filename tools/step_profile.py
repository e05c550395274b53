"""Per-step kernel breakdown of the captured training step (run under rocprofv3
--kernel-trace).  Two marker launches (pose6d_pinhole_z_fwd, which the
RGBD-Geometric step never launches)
bracket `--steps` graph replays; tools/trace_window.py then sums every kernel
between them per step.

    rocprofv3 --kernel-trace -d OUT -o run --output-format csv -- python3 tools/step_profile.py
    python tools/trace_window.py OUT/run_kernel_trace.csv --steps 10
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "6d-pose-estimation_amd")]

import torch  # noqa: E402

from bench import synth_batch  # noqa: E402


def marker():
    from pose6d._lib import call, stream
    z = torch.ones(1, device="cuda")
    bbox = torch.zeros(1, 2, device="cuda")
    K = torch.eye(3, device="cuda")
    t = torch.empty(1, 3, device="cuda")
    call("pinhole_z_fwd", z, bbox, K, 0, 1, t, stream())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--model", default="rgbd_geometric")
    ap.add_argument("--eager", action="store_true", help="no hipGraph (PMC counter passes)")
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "f32"])
    ap.add_argument("--attr", default="", help="module.Class.attribute=0|1 set before the trainer is built")
    a = ap.parse_args()
    from models.pose_net_rgbd_geometric import PoseNetRGBDGeometric
    from pose6d.train import RGBDGeometricTrainer
    torch.manual_seed(0)
    dev = torch.device("cuda", 0)
    model = PoseNetRGBDGeometric(pretrained=False).to(dev)
    if a.attr:
        import importlib
        path, val = a.attr.split("=")
        mod, cls, attr = path.rsplit(".", 2)
        setattr(getattr(importlib.import_module(mod), cls), attr, bool(int(val)))
    tr = RGBDGeometricTrainer(model, 32, dtype=torch.bfloat16 if a.dtype == "bf16" else torch.float32)
    data = synth_batch(32, dev, seed=1000)
    if not a.eager:
        tr.capture(data)
    for _ in range(3):
        tr.step(data)
    torch.cuda.synchronize()
    marker()
    for _ in range(a.steps):
        tr.step(data)
    marker()
    torch.cuda.synchronize()
    print("steps", a.steps, "loss", tr.loss.item())


if __name__ == "__main__":
    main()
