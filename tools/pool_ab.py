"""Time the stem pool kernels (bs32 bf16: 112x112x64 -> 56x56x64, 3x3/s2/p1) in a hipGraph,
for A/B timing of two library builds on one box (POSE6D_LIB selects the build).
usage: POSE6D_LIB=... python tools/pool_ab.py"""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "6d-pose-estimation_amd")]

from pose6d._lib import call  # noqa: E402
from pose6d.trunk import DTYPES  # noqa: E402


def main():
    dev, dt = "cuda", DTYPES[torch.bfloat16]
    N, H, W, C, k, s, p = 32, 112, 112, 64, 3, 2, 1
    Ho, Wo = 56, 56
    x = torch.randn(N, H, W, C, device=dev).bfloat16()
    sc = torch.rand(C, device=dev) + 0.5
    sh = torch.randn(C, device=dev)
    y = torch.empty(N, Ho, Wo, C, device=dev, dtype=torch.bfloat16)
    am = torch.empty(N, Ho, Wo, C, device=dev, dtype=torch.uint8)
    dx = torch.empty_like(x)
    st = torch.cuda.Stream()
    res = {}
    for name in ("fwd", "bwd"):
        def launch(sp):
            if name == "fwd":
                call("bn_relu_maxpool_fwd", dt, x, sc, sh, y, am, N, H, W, C, k, s, p, Ho, Wo, sp)
            else:
                call("maxpool_bwd", dt, y, am, dx, N, H, W, C, k, s, p, Ho, Wo, sp)
        with torch.cuda.stream(st):
            launch(st.cuda_stream)
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=st):
                for _ in range(20):
                    launch(st.cuda_stream)
            g.replay()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            best = 1e9
            for _ in range(10):
                e0.record(st)
                g.replay()
                e1.record(st)
                e1.synchronize()
                best = min(best, e0.elapsed_time(e1) * 1000 / 20)
        res[name] = best
    print(os.environ.get("POSE6D_LIB", "default"), " ".join(f"{k} {v:.1f}us" for k, v in res.items()), flush=True)


if __name__ == "__main__":
    main()
