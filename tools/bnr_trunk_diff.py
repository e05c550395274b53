"""Per-parameter gradient difference of the training trunk backward with / without the
BN reduce folded into the data gradients (TrunkEngine.bwd_conv_bn_reduce), fp32 and bf16."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "6d-pose-estimation_amd")]
import torch  # noqa: E402


def main():
    from pose6d.resnet import resnet50_trunk
    from pose6d.trunk import TrunkEngine
    for dtype in (torch.float32, torch.bfloat16):
        torch.manual_seed(0)
        seq = resnet50_trunk(3).cuda().train()
        eng = TrunkEngine(seq, 3)
        eng.set_dtype(dtype)
        g = torch.Generator().manual_seed(4)
        x = torch.randn(4, 3, 96, 96, generator=g).cuda()
        dfeat = torch.randn(4, 2048, generator=g).cuda()
        grads = []
        for fold in (False, True, False):
            eng.bwd_conv_bn_reduce = fold
            gd = {p: torch.zeros_like(p, dtype=torch.float32) for p in seq.parameters()}
            eng.forward(x, True)
            eng.backward(dfeat, lambda p: gd[p])
            torch.cuda.synchronize()
            grads.append(gd)
        rows = []
        for name, p in seq.named_parameters():
            a, b, c = grads[0][p], grads[1][p], grads[2][p]
            rows.append((((a - b).norm() / (a.norm() + 1e-20)).item(), name, a.norm().item(),
                         ((a - c).norm() / (a.norm() + 1e-20)).item()))
        rows.sort(reverse=True)
        print(dtype, "worst 12 (rel diff, name, |g|, rerun diff):")
        for r in rows[:12]:
            print(f"  {r[0]:.3e} {r[1]:<28} {r[2]:.3e} {r[3]:.1e}")
        med = sorted(r[0] for r in rows)[len(rows) // 2]
        print("  median", f"{med:.3e}")


if __name__ == "__main__":
    main()
