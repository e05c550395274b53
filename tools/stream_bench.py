"""Streaming BatchNorm kernels vs torch elementwise ops of the same bytes (graph-replayed,
L2-cold: a 256 MiB write between launches).  Calibrates how far bn_act / bn_bwd_apply sit
from what a plain streaming kernel reaches on this box.

usage: python tools/stream_bench.py"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "6d-pose-estimation_amd")]

import torch  # noqa: E402

from pose6d._lib import call  # noqa: E402

BF16 = 1


def graph_us(fn, flush, reps=20, n=10):
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        for _ in range(2):
            fn()
            flush()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s, capture_error_mode="thread_local"):
            for _ in range(n):
                flush()
                fn()
        gf = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gf, stream=s, capture_error_mode="thread_local"):
            for _ in range(n):
                flush()
    out = []
    for gg in (g, gf):
        torch.cuda.synchronize()
        gg.replay()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            gg.replay()
        torch.cuda.synchronize()
        out.append((time.perf_counter() - t0) / reps / n * 1e6)
    return out[0] - out[1]


def main():
    dev = torch.device("cuda")
    junk = torch.empty(64 << 20, device=dev)          # 256 MiB
    flush = lambda: junk.fill_(1.0)                    # noqa: E731
    for M, C in ((32 * 56 * 56, 256), (32 * 112 * 112, 64), (32 * 28 * 28, 512)):
        y = torch.randn(M, C, device=dev).to(torch.bfloat16)
        res = torch.randn(M, C, device=dev).to(torch.bfloat16)
        out = torch.empty_like(y)
        mask = torch.empty(M * C // 8, dtype=torch.uint8, device=dev)
        sc, sh = torch.rand(C, device=dev), torch.rand(C, device=dev)
        st = lambda: torch.cuda.current_stream().cuda_stream  # noqa: E731
        mb = M * C * 2 / 1e6
        t_act = graph_us(lambda: call("bn_act_fwd_mask", BF16, y, sc, sh, res, None, None, 1, out, mask, M, C, st()),
                         flush)
        t_add = graph_us(lambda: torch.add(y, res, out=out), flush)
        t_cpy = graph_us(lambda: out.copy_(y), flush)
        print(f"M={M} C={C} ({mb:.1f} MB per tensor): bn_act+res+mask {t_act:6.2f} us "
              f"({(3 * mb + mb / 16) / t_act:.2f} TB/s) | torch add {t_add:6.2f} us ({3 * mb / t_add:.2f} TB/s)"
              f" | torch copy {t_cpy:6.2f} us ({2 * mb / t_cpy:.2f} TB/s)", flush=True)


if __name__ == "__main__":
    main()
