"""ms per fused fp32 training step (RGBDGeometricTrainer, bs32, graph-replayed) as one
JSON line -- for build A/B timing (tools/ab_lib.sh --fp32)."""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "6d-pose-estimation_amd")]

import torch  # noqa: E402

from bench import synth_batch  # noqa: E402


def main(steps=20, warmup=5):
    from models.pose_net_rgbd_geometric import PoseNetRGBDGeometric
    from pose6d.train import RGBDGeometricTrainer
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    tr = RGBDGeometricTrainer(PoseNetRGBDGeometric(pretrained=False).to(dev), 32, dtype=torch.float32)
    data = synth_batch(32, dev, seed=1000)
    tr.capture(data)
    for _ in range(warmup):
        tr.step(data)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        tr.step(data)
    torch.cuda.synchronize()
    print(json.dumps({"ms_per_step": round((time.perf_counter() - t0) / steps * 1e3, 4)}))


if __name__ == "__main__":
    main()
