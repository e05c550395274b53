"""The bf16 128x128 / 8-wave LDS-DMA weight gradient (pose6d_tuning_t wgrad_base = 4)
against the default 64x64 plan on every ResNet50 shape it applies to: the same fp32
sums in another order, so within ~1e-5 relative (Frobenius).
usage: python tools/wgrad128_check.py"""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "6d-pose-estimation_amd")]

from pose6d._lib import Tuning, call, query, stream  # noqa: E402
from pose6d.trunk import DTYPES  # noqa: E402
from tools.conv_bench import SHAPES  # noqa: E402


def main():
    B, dtype, dev = 32, torch.bfloat16, "cuda"
    dt = DTYPES[dtype]
    worst = 0.0
    for (H, W, Cin, Cout, k, s, p) in SHAPES:
        K = k * k * Cin
        if Cout % 128 or K % 128 or Cin % 64:
            continue
        Ho, Wo = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
        g = torch.Generator(device=dev).manual_seed(H * 7 + Cin)
        x = torch.randn(B, H, W, Cin, device=dev, generator=g).to(dtype)
        dy = torch.randn(B, Ho, Wo, Cout, device=dev, generator=g).to(dtype)
        out = []
        for tn in (Tuning(), Tuning(wgrad_base=4)):
            need = query("conv2d_wgrad_workspace_tuned", dt, B, Ho, Wo, Cin, Cout, k, k, tn.ref)
            ws = torch.empty(max(need, 4) // 4 + 1, device=dev)
            dw = torch.full((Cout, Cin, k, k), float("nan"), device=dev)
            call("conv2d_wgrad_tuned", dt, x, dy, dw, 0, ws, ws.numel() * 4, B, H, W, Cin, Cin, Cout, k, k, s, p,
                 Ho, Wo, tn.ref, stream())
            out.append(dw)
        torch.cuda.synchronize()
        a, b = out[0].double(), out[1].double()
        err = ((a - b).norm() / a.norm()).item()
        worst = max(worst, err)
        print(f"{H}x{W} {Cin}->{Cout} k{k}s{s}: rel {err:.2e} finite {bool(torch.isfinite(b).all())}", flush=True)
        assert torch.isfinite(b).all() and err < 1e-5, err
    print("worst", worst)


if __name__ == "__main__":
    main()
