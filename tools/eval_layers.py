"""Per-launch in-step times of the bs32 bf16 eval forward (bench.py's
forward_roofline_eval graph) through pose6d.steptime: one line per kernel with its
conv geometry, us and TFLOP/s.  usage: python tools/eval_layers.py [B] [dtype]"""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "6d-pose-estimation_amd")]

from bench import _time_fn, synth_batch  # noqa: E402
from models.pose_net_rgbd_geometric import PoseNetRGBDGeometric  # noqa: E402
from pose6d import steptime  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
    dt = torch.bfloat16 if (len(sys.argv) < 3 or sys.argv[2] == "bf16") else torch.float32
    dev = torch.device("cuda")
    torch.manual_seed(0)
    m = PoseNetRGBDGeometric(pretrained=False).to(dev).set_compute_dtype(dt).eval()
    b = synth_batch(B, dev, seed=1)
    args = (b[0], None, b[1], b[2], b[3])
    with torch.no_grad():
        m(*args)
        g = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            m(*args)
        torch.cuda.current_stream().wait_stream(s)
        with torch.cuda.graph(g):
            m(*args)
        plain = _time_fn(g.replay, 50) * 1e3
        t = steptime.StepTimer(lambda: m(*args), dev)
        recs = t.run(20, plain_ms=plain)
    print(f"# eval forward B={B} {dt}: {plain:.4f} ms/batch replayed, {len(recs)} kernels, event overhead "
          f"{t.overhead_us:.2f} us/node subtracted")
    tot = 0.0
    for r in recs:
        tf = f"{r['flops'] / (r['us'] * 1e-6) / 1e12:7.1f} TF" if r["flops"] and r["us"] > 0 else ""
        tot += r["us"]
        print(f"{r['us']:8.2f} us  {tf:10s}  {(r['geom'] or ''):24s} {r['kernel'][:70]}")
    print(f"# sum {tot / 1e3:.4f} ms")


if __name__ == "__main__":
    main()
