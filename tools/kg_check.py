"""K-group tile (6) vs the 4-wave 64x64 tile (3) on every ResNet50 forward shape: the
outputs and BN statistics must agree to fp32 summation-order rounding.
usage: python tools/kg_check.py [bf16|f32]"""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "6d-pose-estimation_amd"), os.path.join(REPO, "tools")]

from conv_bench import SHAPES  # noqa: E402
from pose6d._lib import call, query, stream  # noqa: E402
from pose6d.trunk import DTYPES, pack_single  # noqa: E402


def main():
    dtype = torch.bfloat16 if (len(sys.argv) < 2 or sys.argv[1] == "bf16") else torch.float32
    dt, B, dev = DTYPES[dtype], 32, "cuda"
    worst = 0.0
    for (H, W, Cin, Cout, k, s, p) in SHAPES[1:]:
        Ho, Wo = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
        x = torch.randn(B, H, W, Cin, device=dev).to(dtype)
        w = torch.randn(Cout, Cin, k, k, device=dev) * 0.05
        wp, _ = pack_single(w, Cin, dtype)
        rows = query("conv_stats_rows", B, Ho, Wo, Cout)
        outs = {}
        for t in ("3", "6"):
            os.environ["POSE6D_CONV_TILE"] = t
            y = torch.empty(B, Ho, Wo, Cout, device=dev, dtype=dtype)
            st = torch.zeros(2, Cout, rows, device=dev)
            call("conv2d_fwd", dt, x, wp, None, y, st, B, H, W, Cin, Cout, k, k, s, p, Ho, Wo, stream())
            torch.cuda.synchronize()
            outs[t] = (y.float(), st)
        os.environ.pop("POSE6D_CONV_TILE", None)
        dy = (outs["3"][0] - outs["6"][0]).abs().max().item() / outs["3"][0].abs().max().item()
        ds = (outs["3"][1] - outs["6"][1]).abs().max().item() / outs["3"][1].abs().max().item()
        worst = max(worst, dy, ds)
        print(f"{H:3d}x{W:<3d} {Cin:4d}->{Cout:<4d} k{k}s{s}  out rel {dy:.2e}  stats rel {ds:.2e}", flush=True)
    print("worst", worst)
    assert worst < (2e-2 if dtype == torch.bfloat16 else 1e-5), worst


if __name__ == "__main__":
    main()
