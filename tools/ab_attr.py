"""Interleaved A/B of an engine class attribute on the captured bf16 training step:
two trainers (attribute off / on at capture), graph replays alternated in rounds,
median ms per step of each.

    python tools/ab_attr.py pose6d.trunk.TrunkEngine.bwd_dual_bn [--rounds 7 --steps 20]
    python tools/ab_attr.py none      # one trainer, as configured (runtime env A/B across processes)
    python tools/ab_attr.py kw:pack_in_adamw [--dtype f32]   # a trainer keyword False / True
"""
import argparse
import importlib
import os
import statistics
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "6d-pose-estimation_amd")]

import torch  # noqa: E402

from bench import synth_batch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("attr", help="module.Class.attribute")
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "f32"])
    a = ap.parse_args()
    dtype = torch.bfloat16 if a.dtype == "bf16" else torch.float32
    klass, kw = None, None
    if a.attr.startswith("kw:"):
        kw = a.attr[3:]
    elif a.attr != "none":
        mod, cls, attr = a.attr.rsplit(".", 2)
        klass = getattr(importlib.import_module(mod), cls)
    from models.pose_net_rgbd_geometric import PoseNetRGBDGeometric
    from pose6d.train import RGBDGeometricTrainer
    dev = torch.device("cuda", 0)
    data = synth_batch(32, dev, seed=1000)
    trs = {}
    for val in ((False, True) if (klass or kw) else (True,)):
        if klass:
            setattr(klass, attr, val)
        torch.manual_seed(0)
        tr = RGBDGeometricTrainer(PoseNetRGBDGeometric(pretrained=False).to(dev), 32, dtype=dtype,
                                  **({kw: val} if kw else {}))
        tr.capture(data)
        for _ in range(3):
            tr.step(data)
        trs[val] = tr
    torch.cuda.synchronize()
    times = {v: [] for v in trs}
    for _ in range(a.rounds):
        for val, tr in trs.items():
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.steps):
                tr.step(data)
            torch.cuda.synchronize()
            times[val].append((time.perf_counter() - t0) * 1e3 / a.steps)
    for val in trs:
        print(f"{a.attr}={val}: median {statistics.median(times[val]):.4f} ms/step  "
              f"all {[round(t, 4) for t in times[val]]}")
    print("loss", {v: float(t.loss) for v, t in trs.items()})


if __name__ == "__main__":
    main()
