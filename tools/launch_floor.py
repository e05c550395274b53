"""Per-launch floor of a replayed hipGraph on this GPU: N back-to-back launches of a
one-block kernel (pose6d_rownorm_fwd on a 1x4 tensor) captured into one graph.
usage: python tools/launch_floor.py"""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "6d-pose-estimation_amd")]

from pose6d._lib import call, stream  # noqa: E402


def main():
    x = torch.randn(1, 4, device="cuda")
    y = torch.empty_like(x)
    n = 400
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        call("rownorm_fwd", x, y, 1, 4, 0, stream())
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(n):
            call("rownorm_fwd", x, y, 1, 4, 0, stream())
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        g.replay()
    e1.record()
    e1.synchronize()
    print(f"{e0.elapsed_time(e1) / 10 / n * 1e3:.2f} us per launch ({n} one-block launches per graph)")


if __name__ == "__main__":
    main()
