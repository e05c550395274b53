"""Calibration (GPU box): the 1x1 convs of a bs32 ResNet50 step are plain GEMMs, so
torch.mm (hipBLASLt) on the same shapes says what a library GEMM reaches there --
next to our kernels' times for the same convs (forward, data gradient, weight
gradient, fused backward), all graph-replayed.  Not product code.
usage: python tools/gemm_calib.py [--B 32]"""
import argparse
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "6d-pose-estimation_amd")]

from pose6d._lib import call, query, stream  # noqa: E402
from pose6d.trunk import DTYPES, pack_single  # noqa: E402

# (HxW, Cin, Cout) of the distinct stride-1 1x1 convs
SHAPES = [(56, 64, 64), (56, 64, 256), (56, 256, 64), (56, 256, 128), (28, 128, 512), (28, 512, 128),
          (28, 512, 256), (14, 256, 1024), (14, 1024, 256), (14, 1024, 512), (7, 512, 2048), (7, 2048, 512)]


def gtime(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5):
        g.replay()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / (5 * reps) * 1e3   # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=32)
    a = ap.parse_args()
    B, dev, dtype = a.B, "cuda", torch.bfloat16
    dt = DTYPES[dtype]
    print(f"{'shape':>20} | {'mm fwd':>14} {'ours fwd':>14} | {'mm dgrad':>14} {'ours dgrad':>14} | "
          f"{'mm wgrad':>14} {'ours wgrad':>14} | {'ours bwd':>9}")
    for (H, Cin, Cout) in SHAPES:
        M = B * H * H
        fl = 2.0 * M * Cin * Cout
        x = torch.randn(M, Cin, device=dev, dtype=dtype)
        w = torch.randn(Cout, Cin, device=dev, dtype=dtype)
        dy = torch.randn(M, Cout, device=dev, dtype=dtype)
        yo = torch.empty(M, Cout, device=dev, dtype=dtype)
        dxo = torch.empty(M, Cin, device=dev, dtype=dtype)
        dwo = torch.empty(Cout, Cin, device=dev, dtype=dtype)
        wt = w.t()
        t_mm_f = gtime(lambda: torch.mm(x, wt, out=yo))
        t_mm_d = gtime(lambda: torch.mm(dy, w, out=dxo))
        t_mm_w = gtime(lambda: torch.mm(dy.t(), x, out=dwo))
        wp, wtp = pack_single(w.float().view(Cout, Cin, 1, 1), Cin, dtype)
        stats = torch.empty(query("conv_stats_rows", B, H, H, Cout), 2, Cout, device=dev)
        ws = torch.empty(query("conv2d_wgrad_workspace", dt, B, H, H, Cin, Cout, 1, 1) // 4 + 1, device=dev)
        dwf = torch.empty(Cout, Cin, 1, 1, device=dev)
        skw = torch.zeros(64 << 20, device=dev, dtype=torch.uint8)   # split-K workspace (caller-provided)
        t_f = gtime(lambda: call("conv2d_fwd", dt, x, wp, None, yo, stats, B, H, H, Cin, Cout, 1, 1, 1, 0, H, H,
                                 skw, skw.numel(), stream()))
        t_d = gtime(lambda: call("conv2d_dgrad", dt, dy, wtp, None, dxo, B, H, H, Cin, Cout, 1, 1, 1, 0, H, H,
                                 stream()))
        t_w = gtime(lambda: call("conv2d_wgrad", dt, x, dy, dwf, 0, ws, ws.numel() * 4, B, H, H, Cin, Cin, Cout, 1,
                                 1, 1, 0, H, H, stream()))
        wsb = torch.empty(query("conv2d_wgrad_workspace", dt, B, H, H, Cin, Cout, 1, 1) // 4 + 1, device=dev)
        t_b = gtime(lambda: call("conv2d_backward", dt, x, dy, wtp, None, dxo, dwf, 0, wsb, wsb.numel() * 4, B, H, H,
                                 Cin, Cin, Cout, 1, 1, 1, 0, H, H, stream()))

        def f(t):
            return f"{t:6.1f}us/{fl / t / 1e6:5.0f}T"
        print(f"{H:2d}x{H:<2d} {Cin:4d}->{Cout:<4d} M={M:6d} | {f(t_mm_f)} {f(t_f)} | {f(t_mm_d)} {f(t_d)} | "
              f"{f(t_mm_w)} {f(t_w)} | {t_b:6.1f}us", flush=True)


if __name__ == "__main__":
    main()
