"""Time the trainer's optimizer launches (clip partials + AdamW [+ packed weights]) on
the bs32 RGBDGeometric arena: graph of 10 optimizer calls, replayed.
usage: python tools/adamw_bench.py [--dtype f32]   (POSE6D_LIB selects a library build)"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "6d-pose-estimation_amd")]

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "f32"])
    a = ap.parse_args()
    from models.pose_net_rgbd_geometric import PoseNetRGBDGeometric
    from pose6d.train import RGBDGeometricTrainer
    dev = torch.device("cuda")
    dtype = torch.bfloat16 if a.dtype == "bf16" else torch.float32
    for packed in (False, True):
        torch.manual_seed(0)
        tr = RGBDGeometricTrainer(PoseNetRGBDGeometric(pretrained=False).to(dev), 32, dtype=dtype,
                                  pack_in_adamw=packed)
        tr.arena.grad.normal_(0, 1e-3)

        def body():
            tr._pack()
            tr._optimizer()

        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            body()
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(10):
                body()
        g.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ts = []
        for _ in range(5):
            e0.record()
            g.replay()
            e1.record()
            e1.synchronize()
            ts.append(e0.elapsed_time(e1) * 100)   # us per optimizer call
        print(f"pack_in_adamw={packed}: {sorted(ts)[2]:.1f} us per pack + optimizer (all {[round(t, 1) for t in ts]})",
              flush=True)


if __name__ == "__main__":
    main()
