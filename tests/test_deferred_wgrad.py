"""Deferred weight gradients (bf16): each conv's data gradient alone
(pose6d_conv2d_dgrad_ex: the fused launch's data-gradient plan) and the weight
gradients of up to POSE6D_WGRAD_BATCH_MAX convs in one batched launch + one batched
reduce (pose6d_conv2d_wgrad_batch) -- bit-identical to the fused per-conv launches."""
import copy
import ctypes
import warnings

import pytest
import torch

pytestmark = pytest.mark.gpu


def _nhwc(t, cpad=None):
    t = t.permute(0, 2, 3, 1).contiguous()
    if cpad is not None and cpad > t.shape[-1]:
        t = torch.nn.functional.pad(t, (0, cpad - t.shape[-1]))
    return t


SHAPES = [  # N, H, W, Cin(real), Cout, k, s, p
    (2, 14, 14, 256, 64, 1, 1, 0),     # 1x1, several splits
    (2, 7, 7, 512, 128, 1, 1, 0),      # 1x1, one split: dW written directly
    (2, 14, 14, 64, 64, 3, 1, 1),      # 3x3
    (2, 28, 28, 128, 256, 1, 2, 0),    # 1x1 stride 2
    (2, 32, 32, 3, 64, 7, 2, 3),       # the row-tap stem
    (2, 15, 15, 128, 128, 3, 2, 1),    # 3x3 stride 2, odd extent
]


def test_wgrad_batch_matches_single_launches():
    from pose6d._lib import DT_BF16, call, query, stream
    from pose6d.trunk import _WgradJob
    g = torch.Generator().manual_seed(9)
    dev, dtype = "cuda", torch.bfloat16
    jobs, refs, keep = [], [], []
    for i, (N, H, W, Cin, Cout, k, s, p) in enumerate(SHAPES):
        cp = 4 if Cin < 8 else Cin
        Ho, Wo = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
        x = _nhwc(torch.randn(N, Cin, H, W, generator=g), cp).to(dev, dtype)
        dy = torch.randn(N, Ho, Wo, Cout, generator=g).to(dev, dtype)
        acc = i % 2   # written and accumulated jobs
        n = query("conv2d_wgrad_workspace", DT_BF16, N, Ho, Wo, cp, Cout, k, k)
        ws1 = torch.zeros(max(n // 4, 1), device=dev)
        ws2 = torch.zeros(max(n // 4, 1), device=dev)
        init = torch.randn(Cout, Cin, k, k, generator=g).to(dev)
        dw1, dw2 = init.clone(), init.clone()
        call("conv2d_wgrad", DT_BF16, x, dy, dw1, acc, ws1, ws1.numel() * 4, N, H, W, cp, Cin, Cout, k, k, s, p, Ho,
             Wo, stream())
        jobs.append(_WgradJob(x.data_ptr(), dy.data_ptr(), dw2.data_ptr(), ws2.data_ptr(), ws2.numel() * 4, N, H, W,
                              cp, Cin, Cout, k, k, s, p, Ho, Wo, acc))
        refs.append((dw1, dw2))
        keep += [x, dy, ws1, ws2]
    arr = (_WgradJob * len(jobs))(*jobs)
    call("conv2d_wgrad_batch", DT_BF16, ctypes.addressof(arr), len(jobs), stream())
    torch.cuda.synchronize()
    for i, (a, b) in enumerate(refs):
        assert torch.equal(a, b), f"job {i} {SHAPES[i]}: batched dW differs"


def _pair(B):
    from models.pose_net_rgbd_geometric import PoseNetRGBDGeometric
    from pose6d.train import RGBDGeometricTrainer
    warnings.simplefilter("ignore")
    torch.manual_seed(0)
    m0 = PoseNetRGBDGeometric(pretrained=False)
    return [RGBDGeometricTrainer(copy.deepcopy(m0).cuda(), B, dtype=torch.bfloat16) for _ in range(2)]


@pytest.mark.parametrize("B", [4, 32])
def test_trainer_deferred_wgrad_bit_identical(B):
    """Graph-replayed bf16 training steps with the deferred, batched weight gradients equal
    the per-conv fused launches bit for bit (masters, moments, gradients)."""
    from bench import synth_batch
    trs = _pair(B)
    trs[1].trunk.defer_wgrad = True
    data = synth_batch(B, torch.device("cuda"), seed=21)
    for t in trs:
        s = t.snapshot()
        t.capture(data, warmup=1)
        t.restore(s)
    for step in range(2):
        for t in trs:
            t.step()
        torch.cuda.synchronize()
        a, b = trs
        assert torch.equal(a.arena.grad, b.arena.grad), f"step {step}: gradients differ"
        assert torch.equal(a.arena.flat, b.arena.flat), f"step {step}: masters differ"
        assert torch.equal(a.m, b.m) and torch.equal(a.v, b.v), f"step {step}: moments differ"
