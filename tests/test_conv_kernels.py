"""Per-kernel numerics of the conv / BN / pool kernels through the C ABI, against a
plain torch-CPU fp32 reference of the same op (fp32 kernels: 1e-4 relative;
bf16 kernels: against the fp32 op on bf16-rounded operands, bf16 tolerance)."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

CONFIGS = [
    # N, H, W, Cin, Cout, k, s, p, bias
    (2, 14, 14, 64, 128, 1, 1, 0, False),    # 1x1 (GEMM mode), M not a tile multiple
    (2, 28, 28, 256, 512, 1, 2, 0, False),   # downsample 1x1/s2
    (2, 14, 14, 64, 64, 3, 1, 1, False),     # bottleneck 3x3
    (2, 28, 28, 128, 128, 3, 2, 1, False),   # stride-2 3x3
    (2, 15, 15, 128, 64, 3, 2, 1, False),    # stride-2 3x3, odd extent (no parity-class split)
    (2, 32, 32, 3, 64, 7, 2, 3, False),      # stem 7x7/s2, Cin 3 padded to 4
    (2, 16, 16, 32, 64, 5, 1, 2, True),      # z-CNN 5x5 (+bias)
    (2, 32, 32, 3, 32, 7, 2, 3, True),       # z-CNN stem, Cout 32 (+bias)
    (1, 7, 7, 512, 2048, 1, 1, 0, False),    # layer4 expand
]


def _close(got, ref, rtol, what):
    got = got.float().cpu()
    ref = ref.float().cpu()
    scale = ref.abs().max().item() + 1e-30
    err = (got - ref).abs()
    bad = err > (rtol * ref.abs() + rtol * scale)
    assert not bool(bad.any()), f"{what}: max err {err.max().item():.3e} (scale {scale:.3e}), {int(bad.sum())} bad"


def test_s2_class_order_rotation():
    """The stride-2 data gradient's workgroup -> (tile, parity class) map (conv_igemm.hip,
    POSE6D_S2_ROTATE): logical ids 4t .. 4t+3 are tile t's four classes (a permutation,
    so every output pixel is written exactly once, as before), and the class at each
    position mod 4 -- the shader engine a dispatch round-robin hands it to -- rotates
    with t, so every position sees each class equally often."""
    T = 200
    bid = np.arange(4 * T)
    cls = 3 - ((bid + (bid >> 2)) & 3)
    tile = bid >> 2
    for t in range(T):
        assert sorted(cls[tile == t].tolist()) == [0, 1, 2, 3]
    for pos in range(4):
        counts = np.bincount(cls[bid % 4 == pos], minlength=4)
        assert counts.min() == counts.max() == T // 4


_SKWS = {}


def skws(i=0):
    """A zeroed split-K workspace (pose6d_conv_splitk_workspace; 64 MiB covers every
    plan these tests force): (tensor, bytes) for the conv entry points."""
    if i not in _SKWS:
        _SKWS[i] = torch.zeros(64 << 20, device="cuda", dtype=torch.uint8)
    return _SKWS[i], _SKWS[i].numel()


def _nhwc(t, cpad=None):
    t = t.permute(0, 2, 3, 1).contiguous()
    if cpad is not None and cpad > t.shape[-1]:
        t = F.pad(t, (0, cpad - t.shape[-1]))
    return t


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("cfg", CONFIGS)
def test_conv_fwd_dgrad_wgrad(cfg, dtype):
    from pose6d._lib import call, query, stream
    from pose6d.trunk import DTYPES, pack_single
    N, H, W, Cin, Cout, k, s, p, has_bias = cfg
    g = torch.Generator().manual_seed(hash(cfg) & 0xFFFF)
    x = torch.randn(N, Cin, H, W, generator=g)
    w = torch.randn(Cout, Cin, k, k, generator=g) * (2.0 / (Cin * k * k)) ** 0.5
    b = torch.randn(Cout, generator=g) if has_bias else None
    if dtype == torch.bfloat16:   # the reference sees the same rounded operands
        x = x.bfloat16().float()
        w = w.bfloat16().float()
    Ho, Wo = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
    cpad = 4 if Cin < 8 else Cin
    dt = DTYPES[dtype]
    dev = "cuda"
    xd = _nhwc(x, cpad).to(dev, dtype)
    wd = w.to(dev)
    wp, wt = pack_single(wd, cpad, dtype, with_t=Cin >= 8, stride=s, pad=p)
    y = torch.empty(N, Ho, Wo, Cout, device=dev, dtype=dtype)
    rows = query("conv_stats_rows", N, Ho, Wo, Cout)
    stats = torch.empty(2, Cout, rows, device=dev)
    call("conv2d_fwd", dt, xd, wp, b.to(dev) if b is not None else None, y, stats, N, H, W, cpad, Cout, k, k, s, p,
         Ho, Wo, *skws(), stream())
    xr = x.clone().requires_grad_(True)
    wr = w.clone().requires_grad_(True)
    yr = F.conv2d(xr, wr, b, stride=s, padding=p)
    tol = 1e-4 if dtype == torch.float32 else 2e-2
    _close(y.permute(0, 3, 1, 2), yr.detach(), tol, "fwd")
    # epilogue statistics -> finalize: batch mean / biased variance of the fp32 accumulators
    C = Cout
    one, zero = torch.ones(C, device=dev), torch.zeros(C, device=dev)
    rm, rv = torch.zeros(C, device=dev), torch.ones(C, device=dev)
    sc, sh, mu, iv = (torch.empty(C, device=dev) for _ in range(4))
    ws = torch.empty(64 * 3 * C, device=dev, dtype=torch.float64)
    call("bn_finalize", stats, rows, C, N * Ho * Wo, one, zero, rm, rv, None, 0.1, 1e-5, 1, sc, sh, mu, iv, ws,
         stream())
    ref = yr.detach().double()
    _close(mu, ref.mean((0, 2, 3)), 1e-4 if dtype == torch.float32 else 1e-2, "batch mean")
    var = 1.0 / iv.double().cpu() ** 2 - 1e-5
    _close(var, ref.var((0, 2, 3), unbiased=False), 1e-4 if dtype == torch.float32 else 1e-2, "batch var")

    dy = torch.randn(N, Cout, Ho, Wo, generator=g)
    if dtype == torch.bfloat16:
        dy = dy.bfloat16().float()
    yr.backward(dy)
    dyd = _nhwc(dy).to(dev, dtype)
    if Cin >= 8:
        dres = torch.randn(N, H, W, Cin, generator=g).to(dev, dtype)
        dx = torch.empty(N, H, W, Cin, device=dev, dtype=dtype)
        call("conv2d_dgrad", dt, dyd, wt, dres, dx, N, H, W, Cin, Cout, k, k, s, p, Ho, Wo, stream())
        _close(dx.permute(0, 3, 1, 2), xr.grad + dres.float().cpu().permute(0, 3, 1, 2), tol, "dgrad(+res)")
    ws = torch.empty(query("conv2d_wgrad_workspace", dt, N, Ho, Wo, cpad, Cout, k, k) // 4 + 1, device=dev)
    dw = torch.full((Cout, Cin, k, k), 7.0, device=dev)
    call("conv2d_wgrad", dt, xd, dyd, dw, 0, ws, ws.numel() * 4, N, H, W, cpad, Cin, Cout, k, k, s, p, Ho, Wo,
         stream())
    _close(dw, wr.grad, tol, "wgrad")
    dw2 = dw.clone()
    call("conv2d_wgrad", dt, xd, dyd, dw2, 1, ws, ws.numel() * 4, N, H, W, cpad, Cin, Cout, k, k, s, p, Ho, Wo,
         stream())
    _close(dw2, 2 * wr.grad, tol, "wgrad accumulate")
    if has_bias:
        db = torch.empty(Cout, device=dev)
        call("channel_sum", dt, dyd, N * Ho * Wo, Cout, db, 0, stream())
        _close(db, dy.sum((0, 2, 3)), tol, "bias grad")


FAST_CONFIGS = [
    (2, 14, 14, 64, 128, 1, 1, 0),    # GEMM mode
    (2, 14, 14, 64, 64, 3, 1, 1),     # 3x3 implicit GEMM
    (2, 28, 28, 128, 128, 3, 2, 1),   # 3x3/s2: parity-class dgrad
    (2, 28, 28, 256, 512, 1, 2, 0),   # 1x1/s2: parity classes with zero taps
]


@pytest.mark.gpu
@pytest.mark.parametrize("cfg", FAST_CONFIGS)
def test_conv_fast_variants_bit_identical(cfg):
    """Every LDS-ring depth / tile of the bf16 fast path (and the parity-class
    stride-2 dgrad vs the masked gather) accumulates each output in the same K
    order, so all of them must agree bit for bit.  The plans are forced through
    pose6d_tuning_t (the *_tuned entry points); the product calls take none."""
    from pose6d._lib import Tuning, call, query, stream
    from pose6d.trunk import DTYPES, pack_single
    N, H, W, Cin, Cout, k, s, p = cfg
    g = torch.Generator().manual_seed(7)
    dev, dtype = "cuda", torch.bfloat16
    Ho, Wo = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
    x = torch.randn(N, H, W, Cin, generator=g).to(dev, dtype)
    w = (torch.randn(Cout, Cin, k, k, generator=g) * 0.05).to(dev)
    dy = torch.randn(N, Ho, Wo, Cout, generator=g).to(dev, dtype)
    dres = torch.randn(N, H, W, Cin, generator=g).to(dev, dtype)
    wp, wt = pack_single(w, Cin, dtype)
    dt = DTYPES[dtype]
    base = Tuning(wgrad_base=1)
    ws = torch.empty(max(query("conv2d_wgrad_workspace", dt, N, Ho, Wo, Cin, Cout, k, k),
                         query("conv2d_wgrad_workspace_tuned", dt, N, Ho, Wo, Cin, Cout, k, k, base.ref)) // 4 + 1,
                     device=dev)

    def run(tn=None):
        tn = tn if tn is not None else Tuning(conv_patch=0)
        y = torch.empty(N, Ho, Wo, Cout, device=dev, dtype=dtype)
        dx = torch.empty(N, H, W, Cin, device=dev, dtype=dtype)
        dw = torch.empty(Cout, Cin, k, k, device=dev)
        call("conv2d_fwd_tuned", dt, x, wp, None, y, None, N, H, W, Cin, Cout, k, k, s, p, Ho, Wo, tn.ref, *skws(),
             stream())
        call("conv2d_dgrad_tuned", dt, dy, wt, dres, dx, N, H, W, Cin, Cout, k, k, s, p, Ho, Wo, tn.ref, *skws(),
             stream())
        call("conv2d_wgrad_tuned", dt, x, dy, dw, 0, ws, ws.numel() * 4, N, H, W, Cin, Cin, Cout, k, k, s, p, Ho, Wo,
             tn.ref, stream())
        torch.cuda.synchronize()
        return y.cpu(), dx.cpu(), dw.cpu()

    y0, dx0, dw0 = run()
    # the plain (untuned) entry points are the default plan (a stats-free 3x3 stride-1
    # forward takes the patch kernel: its own K order, compared in test_conv3x3_patch)
    y = torch.empty(N, Ho, Wo, Cout, device=dev, dtype=dtype)
    call("conv2d_fwd", dt, x, wp, None, y, None, N, H, W, Cin, Cout, k, k, s, p, Ho, Wo, *skws(), stream())
    torch.cuda.synchronize()
    if query("conv_patch_plan", dt, N, H, W, Cin, Cout, k, k, s, p, Ho, Wo) == 0:
        assert torch.equal(y.cpu(), y0)
    else:
        _close(y.cpu(), y0, 2e-2, "patch plan vs implicit GEMM")
    variants = [dict(conv_stages=st, conv_tile=t) for st in (2, 3, 4, 6) for t in (0, 1, 3, 4, 5)]
    variants.append(dict(conv_s2=0))
    variants += [dict(wgrad_stages=st) for st in (2, 3, 4)]
    for kw in variants:
        y1, dx1, dw1 = run(Tuning(conv_patch=0, **kw))
        assert torch.equal(y0, y1), f"fwd differs under {kw}"
        assert torch.equal(dx0, dx1), f"dgrad differs under {kw}"
        assert torch.equal(dw0, dw1), f"wgrad differs under {kw}"
    # the fused data+weight gradient launch must equal the two separate passes bit for bit
    for sep in (False, True):
        dxf = torch.empty(N, H, W, Cin, device=dev, dtype=dtype)
        dwf = torch.empty(Cout, Cin, k, k, device=dev)
        call("conv2d_backward_tuned", dt, x, dy, wt, dres, dxf, dwf, 0, ws, ws.numel() * 4, N, H, W, Cin, Cin, Cout,
             k, k, s, p, Ho, Wo, Tuning(bwd_separate=int(sep)).ref, stream())
        torch.cuda.synchronize()
        assert torch.equal(dxf.cpu(), dx0), f"fused backward dx differs (separate={sep})"
        assert torch.equal(dwf.cpu(), dw0), f"fused backward dw differs (separate={sep})"
    # residual accumulated in place (dres is dx, as the trunk adds the downsample
    # conv's data gradient to conv1's): same bits as the out-of-place sum
    dxi = dres.clone()
    dwi = torch.empty(Cout, Cin, k, k, device=dev)
    call("conv2d_backward", dt, x, dy, wt, dxi, dxi, dwi, 0, ws, ws.numel() * 4, N, H, W, Cin, Cin, Cout, k, k, s, p,
         Ho, Wo, stream())
    dxd = dres.clone()
    call("conv2d_dgrad", dt, dy, wt, dxd, dxd, N, H, W, Cin, Cout, k, k, s, p, Ho, Wo, stream())
    torch.cuda.synchronize()
    assert torch.equal(dxi.cpu(), dx0), "in-place backward dx differs"
    assert torch.equal(dxd.cpu(), dx0), "in-place dgrad differs"
    # the register-staged weight gradient sums the pixels in other splits: close, not equal
    _, _, dwb = run(base)
    _close(dwb, dw0, 1e-5, "wgrad base vs LDS-DMA")
    # the register-staged conv kernels: other K order, close
    yb, dxb, _ = run(Tuning(conv_base=1))
    _close(yb, y0, 2e-2, "fwd base vs LDS-DMA")
    _close(dxb, dx0, 2e-2, "dgrad base vs LDS-DMA")


PATCH_CONFIGS = [
    # N, H, W, Cin, Cout: tiles of R full rows (14x14: 9 + 5, 28x28: 4, 56x56: 2) or of
    # whole images (7x7: 2 per tile; odd N leaves a one-image tile)
    (32, 14, 14, 256, 256),
    (3, 7, 7, 512, 512),
    (2, 28, 28, 128, 128),
    (2, 56, 56, 64, 64),
    (2, 14, 14, 64, 192),
    (1, 5, 9, 128, 64),
]


@pytest.mark.gpu
@pytest.mark.parametrize("cfg", PATCH_CONFIGS)
def test_conv3x3_patch(cfg):
    """The 3x3 / stride-1 patch kernel (stats-free bf16 forwards; the default plan on the
    56x56 stage, forced with conv_patch = 1 elsewhere): against the torch fp32
    conv of the same bf16 operands; close to the implicit-GEMM plan (conv_patch = 0,
    another K order); a repeated launch reproduces its bits; the untuned eval BN-act
    epilogue (pose6d_conv2d_fwd_act) is bit for bit the untuned plain store +
    pose6d_bn_act_fwd."""
    from pose6d._lib import Tuning, call, query, stream
    from pose6d.trunk import DTYPES, pack_single
    N, H, W, Cin, Cout = cfg
    dtype = torch.bfloat16
    dt = DTYPES[dtype]
    g = torch.Generator().manual_seed(N * 1000 + H * 10 + Cin)
    x = torch.randn(N, Cin, H, W, generator=g).bfloat16().float()
    w = (torch.randn(Cout, Cin, 3, 3, generator=g) * (2.0 / (Cin * 9)) ** 0.5).bfloat16().float()
    b = torch.randn(Cout, generator=g) * 0.1
    default_patch = query("conv_patch_plan", dt, N, H, W, Cin, Cout, 3, 3, 1, 1, H, W) > 0
    assert default_patch == (H * W >= 3136)
    xd = _nhwc(x).to("cuda", dtype)
    wp, _ = pack_single(w.cuda(), Cin, dtype, with_t=False)
    bd = b.cuda()

    def fwd(tn=None, bias=None):
        y = torch.empty(N, H, W, Cout, device="cuda", dtype=dtype)
        if tn is None:
            call("conv2d_fwd", dt, xd, wp, bias, y, None, N, H, W, Cin, Cout, 3, 3, 1, 1, H, W, *skws(), stream())
        else:
            call("conv2d_fwd_tuned", dt, xd, wp, bias, y, None, N, H, W, Cin, Cout, 3, 3, 1, 1, H, W, tn.ref,
                 *skws(), stream())
        torch.cuda.synchronize()
        return y.cpu()

    ref = F.conv2d(x, w, None, stride=1, padding=1)
    for st in (2, 3, 4):
        y = fwd(Tuning(conv_patch=1, conv_stages=st))
        _close(y.permute(0, 3, 1, 2), ref, 2e-2, f"patch fwd ({st} slots)")
        assert torch.equal(fwd(Tuning(conv_patch=1, conv_stages=st)), y), "repeated launch differs"
        if st == 2:
            y2 = y
        else:
            assert torch.equal(y, y2), "the ring depth changed the patch kernel's bits"
    if default_patch:
        assert torch.equal(fwd(), y2), "the default plan is not the patch kernel"
    yb = fwd(Tuning(conv_patch=1), bias=bd)
    _close(yb.permute(0, 3, 1, 2), ref + b.view(1, -1, 1, 1), 2e-2, "patch fwd + bias")
    yg = fwd(Tuning(conv_patch=0))
    _close(yg, y2, 2e-2, "implicit GEMM vs patch")
    # eval BN-act epilogue == plain store + pose6d_bn_act_fwd, bit for bit (default plans)
    sc = (torch.rand(Cout, generator=g) + 0.5).cuda()
    sh = (torch.randn(Cout, generator=g) * 0.1).cuda()
    fused = torch.empty(N, H, W, Cout, device="cuda", dtype=dtype)
    call("conv2d_fwd_act", dt, xd, wp, bd, fused, N, H, W, Cin, Cout, 3, 3, 1, 1, H, W, sc, sh, None, None, None, 1,
         *skws(), stream())
    plain = fwd(bias=bd)
    sep = torch.empty(N, H, W, Cout, device="cuda", dtype=dtype)
    call("bn_act_fwd", dt, plain.cuda(), sc, sh, None, None, None, 1, sep, N * H * W, Cout, stream())
    torch.cuda.synchronize()
    assert torch.equal(fused.cpu(), sep.cpu()), "BN-act epilogue != conv + bn_act"


SPLITK_CONFIGS = [
    (4, 14, 14, 1024, 256, 1, 1, 0),   # layer3 1x1 reduce (GEMM mode, K = 16 steps)
    (4, 7, 7, 512, 512, 3, 1, 1),      # layer4 3x3 (implicit GEMM, 72 steps, taps split mid-way)
    (2, 14, 14, 256, 256, 3, 2, 1),    # 3x3 / s2 forward (its data gradient: parity classes, not split)
    (3, 7, 7, 2048, 512, 1, 1, 0),     # layer4 1x1 reduce, M = 147 (partial last row tile)
]


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("cfg", SPLITK_CONFIGS)
def test_conv_splitk(cfg, dtype):
    """Split-K inside one launch (pose6d_tuning_t.conv_splitk): each tile's K-steps over
    several workgroups, partials merged by the last arriver in split order.  Against
    the torch fp32 op (forward, BN statistics, data gradient + residual); for one split
    count every tile / ring depth gives the same bits (the sum order depends on the
    split count only), and a repeated launch reproduces them (the arrival counters
    re-arm themselves)."""
    from pose6d._lib import Tuning, call, query, stream
    from pose6d.trunk import DTYPES, pack_single
    N, H, W, Cin, Cout, k, s, p = cfg
    g = torch.Generator().manual_seed(11)
    dev = "cuda"
    Ho, Wo = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
    x = torch.randn(N, Cin, H, W, generator=g)
    w = torch.randn(Cout, Cin, k, k, generator=g) * (2.0 / (Cin * k * k)) ** 0.5
    dy = torch.randn(N, Cout, Ho, Wo, generator=g)
    dres = torch.randn(N, Cin, H, W, generator=g)
    if dtype == torch.bfloat16:
        x, w, dy, dres = (t.bfloat16().float() for t in (x, w, dy, dres))
    xr = x.clone().requires_grad_(True)
    yr = F.conv2d(xr, w, None, stride=s, padding=p)
    yr.backward(dy)
    dt = DTYPES[dtype]
    xd, dyd, dresd = _nhwc(x).to(dev, dtype), _nhwc(dy).to(dev, dtype), _nhwc(dres).to(dev, dtype)
    wp, wt = pack_single(w.to(dev), Cin, dtype)
    rows = query("conv_stats_rows", N, Ho, Wo, Cout)
    tol = 1e-4 if dtype == torch.float32 else 2e-2

    def run(**kw):
        tn = Tuning(**kw)
        y = torch.empty(N, Ho, Wo, Cout, device=dev, dtype=dtype)
        st = torch.empty(2, Cout, rows, device=dev)
        dx = torch.empty(N, H, W, Cin, device=dev, dtype=dtype)
        need = query("conv_splitk_workspace_tuned", dt, 0, N, H, W, Cin, Cout, k, k, s, p, Ho, Wo, tn.ref)
        assert need == 0 or need <= skws()[1]
        call("conv2d_fwd_tuned", dt, xd, wp, None, y, st, N, H, W, Cin, Cout, k, k, s, p, Ho, Wo, tn.ref, *skws(),
             stream())
        call("conv2d_dgrad_tuned", dt, dyd, wt, dresd, dx, N, H, W, Cin, Cout, k, k, s, p, Ho, Wo, tn.ref,
             *skws(), stream())
        torch.cuda.synchronize()
        return y.cpu(), st.cpu(), dx.cpu()

    for splits in (1, 2, 3, 4, 7):
        ref = None
        for tile in (3, 4, 0):
            for stages in (2, 4):
                got = run(conv_splitk=splits, conv_tile=tile, conv_stages=stages)
                if ref is None:
                    ref = got
                    y, st, dx = got
                    _close(y.permute(0, 3, 1, 2), yr.detach(), tol, f"fwd splits={splits}")
                    _close(dx.permute(0, 3, 1, 2), xr.grad + dres, tol, f"dgrad splits={splits}")
                    # the statistics rows of the epilogue: per-32-row sums add up to the column sums
                    ysum = yr.detach().double().sum((0, 2, 3))
                    _close(st[0].double().sum(1), ysum, 1e-3 if dtype == torch.float32 else 2e-2,
                           f"stats sum splits={splits}")
                else:
                    for a, b, what in zip(ref, got, ("fwd", "stats", "dgrad")):
                        assert torch.equal(a, b), f"{what}: splits={splits} tile={tile} stages={stages} differs"
        again = run(conv_splitk=splits)
        for a, b, what in zip(ref, again, ("fwd", "stats", "dgrad")):
            assert torch.equal(a, b), f"{what}: repeated launch differs (splits={splits})"


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_conv_splitk_workspace_contract(dtype):
    """The split-K scratch is the caller's (include/pose6d.h, pose6d_conv_splitk_workspace):
    a plan that splits refuses a missing / short workspace, and split-K forwards running
    CONCURRENTLY on two streams, each with its own workspace, give the serial bits."""
    from pose6d._lib import Pose6dError, call, query
    from pose6d.trunk import DTYPES, pack_single
    dt = DTYPES[dtype]
    shapes = [(32, 7, 7, 512, 512, 3, 1, 1), (32, 7, 7, 2048, 512, 1, 1, 0)]   # layer4: default plans split
    g = torch.Generator().manual_seed(5)
    cases = []
    for N, H, W, Cin, Cout, k, s, p in shapes:
        Ho, Wo = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
        assert query("conv_variant", dt, 0, N, H, W, Cin, Cout, k, k, s, p, Ho, Wo) >> 16 > 1
        need = query("conv_splitk_workspace", dt, 0, N, H, W, Cin, Cout, k, k, s, p, Ho, Wo)
        assert need > 32768
        x = torch.randn(N, H, W, Cin, generator=g).to("cuda", dtype)
        w = (torch.randn(Cout, Cin, k, k, generator=g) * (1.0 / (Cin * k * k)) ** 0.5).cuda()
        wp, _ = pack_single(w, Cin, dtype, with_t=False)
        cases.append(((N, H, W, Cin, Cout, k, k, s, p, Ho, Wo), x, wp, need))
    args, x, wp, need = cases[0]
    y = torch.empty(args[0], args[9], args[10], args[4], device="cuda", dtype=dtype)
    st = ctypes_stream(torch.cuda.current_stream())
    with pytest.raises(Pose6dError, match="split-K workspace"):
        call("conv2d_fwd", dt, x, wp, None, y, None, *args, None, 0, st)
    small = torch.zeros(need - 256, device="cuda", dtype=torch.uint8)
    with pytest.raises(Pose6dError, match="split-K workspace"):
        call("conv2d_fwd", dt, x, wp, None, y, None, *args, small, small.numel(), st)

    def run_all(streams, wss, reps):
        torch.cuda.synchronize()
        outs = [[torch.empty(a[0], a[9], a[10], a[4], device="cuda", dtype=dtype) for _ in range(reps)]
                for a, _, _, _ in cases]
        for r in range(reps):
            for i, (a, xx, ww, _) in enumerate(cases):
                sidx = (i + r) % len(streams)
                with torch.cuda.stream(streams[sidx]):
                    call("conv2d_fwd", dt, xx, ww, None, outs[i][r], None, *a, wss[sidx], wss[sidx].numel(),
                         ctypes_stream(streams[sidx]))
        torch.cuda.synchronize()
        return [[o.cpu() for o in row] for row in outs]

    big = max(c[3] for c in cases)
    ws_a = torch.zeros(big, device="cuda", dtype=torch.uint8)
    ws_b = torch.zeros(big, device="cuda", dtype=torch.uint8)
    serial = run_all([torch.cuda.current_stream()], [ws_a], 1)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    conc = run_all([s1, s2], [ws_a, ws_b], 6)
    for i in range(len(cases)):
        for r in range(6):
            assert torch.equal(conc[i][r], serial[i][0]), f"shape {i} rep {r}: concurrent split-K differs"
    # the counters are left zero (re-armed by every launch)
    assert int(ws_a[:32768].count_nonzero()) == 0 and int(ws_b[:32768].count_nonzero()) == 0


def ctypes_stream(s):
    import ctypes
    return ctypes.c_void_p(s.cuda_stream)


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("C,N,H", [(64, 4, 9), (32, 2, 7), (256, 8, 33)])
def test_bn_act_and_backward(dtype, C, N, H):
    """BN finalize / apply / backward vs torch; every call is made twice and must
    give identical results (no state carried between calls)."""
    from pose6d._lib import call, query, stream
    from pose6d.trunk import DTYPES
    g = torch.Generator().manual_seed(3)
    W = H
    M = N * H * W
    y = torch.randn(N, C, H, W, generator=g) * 2 + 0.5
    res = torch.randn(N, C, H, W, generator=g)
    if dtype == torch.bfloat16:
        y, res = y.bfloat16().float(), res.bfloat16().float()
    gamma = torch.rand(C, generator=g) + 0.5
    beta = torch.randn(C, generator=g)
    dev, dt = "cuda", DTYPES[dtype]
    # statistics partials as the conv epilogue emits them: per 32 pixels (sum, M2),
    # channel-major [2][C][rows]
    flat = y.permute(0, 2, 3, 1).reshape(M, C).double()
    rows = (M + 31) // 32
    part = torch.zeros(2, C, rows, dtype=torch.float64)
    for r in range(rows):
        blk = flat[32 * r:32 * r + 32]
        part[0, :, r] = blk.sum(0)
        part[1, :, r] = ((blk - blk.mean(0)) ** 2).sum(0)
    stats = part.float().to(dev)
    rm, rv = torch.zeros(C, device=dev), torch.ones(C, device=dev)
    nbt = torch.zeros((), dtype=torch.long, device=dev)
    sc, sh, mu, iv = (torch.empty(C, device=dev) for _ in range(4))
    ws = torch.empty(64 * 3 * C, device=dev, dtype=torch.float64)
    for rep in range(2):
        if rep == 1:
            first = [t.clone() for t in (sc, sh, mu, iv)]
            rm, rv = torch.zeros(C, device=dev), torch.ones(C, device=dev)
            nbt.zero_()
        call("bn_finalize", stats, rows, C, M, gamma.to(dev), beta.to(dev), rm, rv, nbt, 0.1, 1e-5, 1, sc, sh, mu, iv,
             ws, stream())
    for a, b in zip(first, (sc, sh, mu, iv)):
        assert torch.equal(a, b), "bn_finalize not repeatable"
    yd, rd = _nhwc(y).to(dev, dtype), _nhwc(res).to(dev, dtype)
    out = torch.empty_like(yd)
    call("bn_act_fwd", dt, yd, sc, sh, rd, None, None, 1, out, M, C, stream())
    yr = y.clone().requires_grad_(True)
    gr, br = gamma.clone().requires_grad_(True), beta.clone().requires_grad_(True)
    rrm, rrv = torch.zeros(C), torch.ones(C)
    o_ref = F.relu(F.batch_norm(yr, rrm, rrv, gr, br, True, 0.1, 1e-5) + res)
    tol = 1e-5 if dtype == torch.float32 else 1e-2
    _close(out.permute(0, 3, 1, 2), o_ref.detach(), tol * 10, "bn_act")
    _close(rm, rrm, 1e-5, "running_mean")
    _close(rv, rrv, 1e-5, "running_var")
    assert int(nbt.item()) == 1
    dout = torch.randn(N, C, H, W, generator=g)
    if dtype == torch.bfloat16:
        dout = dout.bfloat16().float()
    o_ref.backward(dout)
    ws = torch.empty((query("bn_bwd_workspace_rows", M) * 2 + 3) * C, device=dev)
    dy = torch.empty_like(yd)
    dz = torch.empty_like(yd)
    dg, db = torch.empty(C, device=dev), torch.empty(C, device=dev)
    for rep in range(2):
        call("bn_bwd", dt, _nhwc(dout).to(dev, dtype), out, None, None, yd, mu, iv, gamma.to(dev), dg, db, 0, dy, dz,
             ws, M, C, stream())
        if rep == 0:
            first = [t.clone() for t in (dy, dg, db)]
    for a, b in zip(first, (dy, dg, db)):
        assert torch.equal(a, b), "bn_bwd not repeatable"
    # the same BN without residual: the ReLU mask recomputed from y (no forward output
    # read) must equal the one read from the forward output, bit for bit
    out2 = torch.empty_like(yd)
    call("bn_act_fwd", dt, yd, sc, sh, None, None, None, 1, out2, M, C, stream())
    got = []
    for args in ((out2, None, None), (None, sc, sh)):
        dy2, dz2 = torch.empty_like(yd), torch.empty_like(yd)
        dg2, db2 = torch.empty(C, device=dev), torch.empty(C, device=dev)
        call("bn_bwd", dt, _nhwc(dout).to(dev, dtype), *args, yd, mu, iv, gamma.to(dev), dg2, db2, 0, dy2, dz2, ws, M,
             C, stream())
        got.append((dy2.cpu(), dz2.cpu(), dg2.cpu(), db2.cpu()))
    for a, b in zip(*got):
        assert torch.equal(a, b), "recomputed ReLU mask differs from the stored one"
    _close(dy.permute(0, 3, 1, 2), yr.grad, 1e-4 if dtype == torch.float32 else 3e-2, "bn dy")
    _close(dg, gr.grad, 1e-4 if dtype == torch.float32 else 3e-2, "dgamma")
    _close(db, br.grad, 1e-4 if dtype == torch.float32 else 3e-2, "dbeta")
    mask = (o_ref.detach() > 0).float()
    _close(dz.permute(0, 3, 1, 2), dout * mask, 1e-6, "dz")


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("cfg", [(4, 14, 14, 256, 64, 1, 1, 0), (2, 14, 14, 64, 64, 3, 1, 1)])
def test_backward_masked_residual(cfg, dtype):
    """conv backward whose residual is (dout, ReLU bits) equals the one fed the
    materialised dz = dout * mask (the residual BN backward's dz_out), bit for bit,
    dW included; the bits are pose6d_bn_act_fwd_mask's."""
    import ctypes
    from pose6d._lib import call, query, stream
    from pose6d.trunk import DTYPES, pack_single
    N, H, W, Cin, Cout, k, s, p = cfg
    g = torch.Generator().manual_seed(11)
    dev, dt = "cuda", DTYPES[dtype]
    Ho, Wo = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
    M = N * H * W
    x = _nhwc(torch.randn(N, Cin, H, W, generator=g)).to(dev, dtype)
    w = (torch.randn(Cout, Cin, k, k, generator=g) * 0.05).to(dev)
    _, wt = pack_single(w, Cin, dtype)
    dy = _nhwc(torch.randn(N, Cout, Ho, Wo, generator=g)).to(dev, dtype)
    # the residual BN's forward: out = relu(y * sc + sh + res), bits = out > 0
    yraw = _nhwc(torch.randn(N, Cin, H, W, generator=g)).to(dev, dtype)
    res = _nhwc(torch.randn(N, Cin, H, W, generator=g)).to(dev, dtype)
    sc = (torch.rand(Cin, generator=g) + 0.5).to(dev)
    sh = torch.randn(Cin, generator=g).to(dev)
    out = torch.empty_like(yraw)
    vec = 8 if dtype == torch.bfloat16 else 4
    bits = torch.empty(M * Cin // vec, device=dev, dtype=torch.uint8)
    call("bn_act_fwd_mask", dt, yraw, sc, sh, res, None, None, 1, out, bits, M, Cin, stream())
    dout = _nhwc(torch.randn(N, Cin, H, W, generator=g)).to(dev, dtype)
    dz = torch.where(out > 0, dout, torch.zeros_like(dout))
    ws = torch.empty(query("conv2d_wgrad_workspace", dt, N, Ho, Wo, Cin, Cout, k, k) // 4 + 1, device=dev)
    res_out = []
    for masked in (False, True):
        dx = torch.full_like(x, float("nan"))
        dw = torch.empty(Cout, Cin, k, k, device=dev)
        deferred = ctypes.c_int32(0)
        tail = (dx, dw, 0, ws, ws.numel() * 4, N, H, W, Cin, Cin, Cout, k, k, s, p, Ho, Wo, None,
                ctypes.addressof(deferred), stream())
        if masked:
            call("conv2d_backward_chain_masked", dt, x, dy, wt, dout, bits, *tail)
        else:
            call("conv2d_backward_chain", dt, x, dy, wt, dz, *tail)
        if deferred.value:   # this conv's slab reduce was left for a following launch
            from pose6d.trunk import _WgradReduce
            job = _WgradReduce(ws.data_ptr(), dw.data_ptr(), dt, N, H, W, Cin, Cin, Cout, k, k, s, p, Ho, Wo, 0)
            call("wgrad_reduce", ctypes.addressof(job), stream())
        torch.cuda.synchronize()
        res_out.append((dx.clone(), dw.clone()))
    assert torch.equal(res_out[0][0], res_out[1][0]), "masked residual dX differs"
    assert torch.equal(res_out[0][1], res_out[1][1]), "dW differs"


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("cfg", [(4, 14, 14, 256, 128, 1, 1, 0), (2, 14, 14, 64, 64, 3, 1, 1)])
def test_backward_dispatch_order_and_splits(cfg, dtype):
    """The fused backward's dispatch order (pose6d_tuning_t.bwd_order) changes only which
    workgroups start first: dX and dW bit-identical either way; a forced weight-gradient
    split count (wgrad_splits, tools only) sums the pixels in another order: dW close to
    the default plan's."""
    from pose6d._lib import Tuning, call, query, stream
    from pose6d.trunk import DTYPES, pack_single
    N, H, W, Cin, Cout, k, s, p = cfg
    g = torch.Generator().manual_seed(21)
    dev, dt = "cuda", DTYPES[dtype]
    Ho, Wo = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
    x = _nhwc(torch.randn(N, Cin, H, W, generator=g)).to(dev, dtype)
    w = (torch.randn(Cout, Cin, k, k, generator=g) * 0.05).to(dev)
    _, wt = pack_single(w, Cin, dtype)
    dy = _nhwc(torch.randn(N, Cout, Ho, Wo, generator=g)).to(dev, dtype)
    outs = []
    for tn in (Tuning(bwd_order=0), Tuning(bwd_order=1), Tuning(wgrad_splits=1), Tuning(wgrad_splits=3)):
        ws = torch.empty(query("conv2d_wgrad_workspace_tuned", dt, N, Ho, Wo, Cin, Cout, k, k, tn.ref) // 4 + 1,
                         device=dev)
        dx = torch.full_like(x, float("nan"))
        dw = torch.empty(Cout, Cin, k, k, device=dev)
        call("conv2d_backward_tuned", dt, x, dy, wt, None, dx, dw, 0, ws, ws.numel() * 4, N, H, W, Cin, Cin, Cout, k,
             k, s, p, Ho, Wo, tn.ref, stream())
        torch.cuda.synchronize()
        outs.append((dx.clone(), dw.clone()))
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
    for dx, dw in outs[2:]:
        assert torch.equal(dx, outs[0][0])
        _close(dw.cpu(), outs[0][1].cpu(), 1e-4, f"dW with forced splits {cfg}")


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_backward_chain_carried_reduce(dtype):
    """pose6d_conv2d_backward_chain over three convs as the trunk issues them: each call
    may leave its weight-gradient slab reduce pending (*deferred) for the next call to
    run as trailing workgroups (`prev`, ping-pong workspaces) -- the fp32 LDS-DMA and
    register-staged weight gradients carry it too, and a stem-shaped conv (Cin 4,
    dx = NULL) closes the chain.  dX and dW must equal separate pose6d_conv2d_backward
    calls bit for bit (the reduce is the same launch body, only moved)."""
    import ctypes
    from pose6d._lib import Tuning, call, query, stream
    from pose6d.trunk import DTYPES, _WgradReduce, pack_single
    g = torch.Generator().manual_seed(21)
    dev, dt = "cuda", DTYPES[dtype]
    N = 2
    convs = [  # (H, W, Cin, Cin_real, Cout, k, s, p, has dgrad)
        (14, 14, 256, 256, 256, 3, 1, 1, True),
        (14, 14, 128, 128, 256, 1, 1, 0, True),
        (32, 32, 4, 3, 64, 7, 2, 3, False),
    ]
    ops = []
    wsz = 0
    for (H, W, Cin, Cr, Cout, k, s, p, dg) in convs:
        Ho, Wo = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
        x = torch.randn(N, Cin, H, W, generator=g)
        x[:, Cr:] = 0.0   # the padded input channels (stem: RGB padded to 4)
        x = _nhwc(x).to(dev, dtype)
        w = (torch.randn(Cout, Cr, k, k, generator=g) * 0.05).to(dev)
        wp, wt = pack_single(w, Cin, dtype, with_t=dg)
        dy = _nhwc(torch.randn(N, Cout, Ho, Wo, generator=g)).to(dev, dtype)
        ops.append((H, W, Cin, Cr, Cout, k, s, p, dg, Ho, Wo, x, wt, dy))
        wsz = max(wsz, query("conv2d_wgrad_workspace", dt, N, Ho, Wo, Cin, Cout, k, k))
    # separate calls: the reference -- as one conv2d_backward each, and as data and
    # weight gradient in separate launches (the fused launch must match them bit for bit)
    ref = []
    ws = torch.empty(wsz // 4 + 1, device=dev)
    for (H, W, Cin, Cr, Cout, k, s, p, dg, Ho, Wo, x, wt, dy) in ops:
        outs = []
        for sep in (0, 1):
            dx = torch.empty(N, H, W, Cin, device=dev, dtype=dtype) if dg else None
            dw = torch.empty(Cout, Cr, k, k, device=dev)
            call("conv2d_backward_tuned", dt, x, dy, wt if dg else None, None, dx, dw, 0, ws, ws.numel() * 4, N, H, W,
                 Cin, Cr, Cout, k, k, s, p, Ho, Wo, Tuning(bwd_separate=sep).ref, stream())
            torch.cuda.synchronize()
            outs.append((dx.clone() if dg else None, dw.clone()))
        if dg:
            assert torch.equal(outs[0][0], outs[1][0]), f"fused vs separate dX differ {(H, Cin, Cout, k)}"
        assert torch.equal(outs[0][1], outs[1][1]), f"fused vs separate dW differ {(H, Cin, Cout, k)}"
        ref.append(outs[0])
    # the chain
    ws_pp = (torch.empty(wsz // 4 + 1, device=dev), torch.empty(wsz // 4 + 1, device=dev))
    slot, pending, keep = 0, None, []
    deferred = ctypes.c_int32(0)
    got = []
    for (H, W, Cin, Cr, Cout, k, s, p, dg, Ho, Wo, x, wt, dy) in ops:
        ws = ws_pp[slot]
        dx = torch.full((N, H, W, Cin), float("nan"), device=dev, dtype=dtype) if dg else None
        dw = torch.full((Cout, Cr, k, k), float("nan"), device=dev)
        call("conv2d_backward_chain", dt, x, dy, wt if dg else None, None, dx, dw, 0, ws, ws.numel() * 4, N, H, W,
             Cin, Cr, Cout, k, k, s, p, Ho, Wo, ctypes.addressof(pending) if pending is not None else None,
             ctypes.addressof(deferred), stream())
        got.append((dx, dw))
        if deferred.value:
            pending = _WgradReduce(ws.data_ptr(), dw.data_ptr(), dt, N, H, W, Cin, Cr, Cout, k, k, s, p, Ho, Wo, 0)
            keep.append(pending)
            slot ^= 1
        else:
            pending = None
    if pending is not None:
        call("wgrad_reduce", ctypes.addressof(pending), stream())
    torch.cuda.synchronize()
    for i, ((rdx, rdw), (gdx, gdw)) in enumerate(zip(ref, got)):
        if rdx is not None:
            assert torch.equal(rdx, gdx), f"conv {i}: chained dX differs"
        assert torch.equal(rdw, gdw), f"conv {i}: chained dW differs"


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_wgrad_fast_vs_register_staged(dtype):
    """The LDS-DMA weight gradient (bf16 and, since round 4, fp32 with 64x64 and 128x128
    tiles: Tuning(wgrad_base=2 / 3)) against the register-staged kernel
    (Tuning(wgrad_base=1)) and the torch op: other split plans sum the pixels in another
    order, so close, not equal; a stride-2 3x3, a partial last split and a 1x1 with more
    than one k tile."""
    from pose6d._lib import Tuning, call, query, stream
    from pose6d.trunk import DTYPES
    g = torch.Generator().manual_seed(5)
    dev, dt = "cuda", DTYPES[dtype]
    for (N, H, W, Cin, Cout, k, s, p) in [(2, 28, 28, 128, 128, 3, 2, 1), (3, 15, 15, 64, 128, 3, 1, 1),
                                          (2, 14, 14, 256, 192, 1, 1, 0), (2, 28, 28, 64, 256, 1, 2, 0),
                                          (3, 9, 9, 256, 256, 3, 1, 1), (2, 13, 13, 128, 256, 1, 1, 0)]:
        Ho, Wo = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
        x = torch.randn(N, Cin, H, W, generator=g)
        dyt = torch.randn(N, Cout, Ho, Wo, generator=g)
        if dtype == torch.bfloat16:
            x, dyt = x.bfloat16().float(), dyt.bfloat16().float()
        ref = torch.nn.grad.conv2d_weight(x.double(), (Cout, Cin, k, k), dyt.double(), stride=s, padding=p)
        xd, dyd = _nhwc(x).to(dev, dtype), _nhwc(dyt).to(dev, dtype)
        outs = []
        tunings = [Tuning(), Tuning(wgrad_base=1)]
        if dtype == torch.float32:
            tunings += [Tuning(wgrad_base=2), Tuning(wgrad_base=3)]
        for tn in tunings:
            ws = torch.empty(query("conv2d_wgrad_workspace_tuned", dt, N, Ho, Wo, Cin, Cout, k, k, tn.ref) // 4 + 1,
                             device=dev)
            dw = torch.empty(Cout, Cin, k, k, device=dev)
            call("conv2d_wgrad_tuned", dt, xd, dyd, dw, 0, ws, ws.numel() * 4, N, H, W, Cin, Cin, Cout, k, k, s, p,
                 Ho, Wo, tn.ref, stream())
            torch.cuda.synchronize()
            outs.append(dw.cpu())
        for i, o in enumerate(outs):   # default, register-staged, [fp32 64x64, 128x128]
            _close(o, ref.float(), 1e-4, f"wgrad plan {i} {(H, Cin, Cout, k, s)}")


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("cfg", [(2, 32, 32, 3, 64), (4, 224, 224, 3, 64), (2, 30, 26, 3, 128), (2, 29, 27, 3, 64)])
def test_stem_wgrad_rowtap(cfg, dtype):
    """The 4-channel 7x7 / stride-2 stem's weight gradient on the LDS-DMA body (bf16, and
    the fp32 body: one pixel per 16-byte chunk, so odd widths too) with the row-tap X image (slabs in (kernel row, 8 taps, channel) order, mapped back to OIHW
    by the reduce): against the float64 torch op on the same bf16 operands, and against
    the register-staged kernel (Tuning(wgrad_base=1)); written and accumulated, standalone
    and in chain mode (pose6d_conv2d_backward_chain without a data gradient, carrying a
    previous conv's pending slab reduce and leaving its own pending)."""
    import ctypes
    from pose6d._lib import Tuning, call, query, stream
    from pose6d.trunk import DTYPES, _WgradReduce
    N, H, W, Cin, Cout = cfg
    k, s, p, cp = 7, 2, 3, 4
    dev = "cuda"
    dt = DTYPES[dtype]
    Ho, Wo = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
    g = torch.Generator().manual_seed(N + H + Cout)
    x = torch.randn(N, Cin, H, W, generator=g).bfloat16().float()
    dyt = torch.randn(N, Cout, Ho, Wo, generator=g).bfloat16().float()
    ref = torch.nn.grad.conv2d_weight(x.double(), (Cout, Cin, k, k), dyt.double(), stride=s, padding=p)
    xd, dyd = _nhwc(x, cp).to(dev, dtype), _nhwc(dyt).to(dev, dtype)
    outs = []
    for tn in (Tuning(), Tuning(wgrad_base=1)):
        ws = torch.empty(query("conv2d_wgrad_workspace_tuned", dt, N, Ho, Wo, cp, Cout, k, k, tn.ref) // 4 + 1,
                         device=dev)
        dw = torch.full((Cout, Cin, k, k), 0.5, device=dev)
        call("conv2d_wgrad_tuned", dt, xd, dyd, dw, 1, ws, ws.numel() * 4, N, H, W, cp, Cin, Cout, k, k, s, p,
             Ho, Wo, tn.ref, stream())
        torch.cuda.synchronize()
        outs.append(dw.cpu() - 0.5)
    for i, o in enumerate(outs):
        _close(o, ref.float(), 1e-4, f"stem wgrad plan {i} {cfg}")
    # chain mode: a previous (1x1) conv's pending reduce rides on the stem's launch
    N2, C2 = 2, 64
    x2 = torch.randn(N2, 8, 8, C2, generator=g).to(dev, dtype)
    dy2 = torch.randn(N2, 8, 8, C2, generator=g).to(dev, dtype)
    ws2 = torch.zeros(query("conv2d_wgrad_workspace", dt, N2, 8, 8, C2, C2, 1, 1) // 4 + 1, device=dev)
    dw2 = torch.zeros(C2, C2, 1, 1, device=dev)
    dx2 = torch.empty(N2, 8, 8, C2, device=dev, dtype=dtype)
    deferred = ctypes.c_int32(0)
    wt2 = torch.zeros(C2, 1, 1, C2, device=dev, dtype=dtype)
    call("conv2d_backward_chain", dt, x2, dy2, wt2, None, dx2, dw2, 0, ws2, ws2.numel() * 4, N2, 8, 8, C2, C2, C2, 1,
         1, 1, 0, 8, 8, None, ctypes.addressof(deferred), stream())
    prev = _WgradReduce(ws2.data_ptr(), dw2.data_ptr(), dt, N2, 8, 8, C2, C2, C2, 1, 1, 1, 0, 8, 8, 0)
    ws = torch.empty(query("conv2d_wgrad_workspace", dt, N, Ho, Wo, cp, Cout, k, k) // 4 + 1, device=dev)
    dw = torch.zeros(Cout, Cin, k, k, device=dev)
    d2 = ctypes.c_int32(0)
    call("conv2d_backward_chain", dt, xd, dyd, None, None, None, dw, 0, ws, ws.numel() * 4, N, H, W, cp, Cin, Cout,
         k, k, s, p, Ho, Wo, ctypes.addressof(prev) if deferred.value else None, ctypes.addressof(d2), stream())
    if d2.value:
        job = _WgradReduce(ws.data_ptr(), dw.data_ptr(), dt, N, H, W, cp, Cin, Cout, k, k, s, p, Ho, Wo, 0)
        call("wgrad_reduce", ctypes.addressof(job), stream())
    torch.cuda.synchronize()
    _close(dw.cpu(), ref.float(), 1e-4, f"stem wgrad chain {cfg}")
    ref2 = torch.einsum("nhwc,nhwd->dc", x2.double().cpu(), dy2.double().cpu()).reshape(C2, C2, 1, 1)
    _close(dw2.cpu(), ref2.float(), 1e-4, "carried 1x1 reduce")


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_pools(dtype):
    from pose6d._lib import call, stream
    from pose6d.trunk import DTYPES
    g = torch.Generator().manual_seed(4)
    dev, dt = "cuda", DTYPES[dtype]
    # stem 3x3/s2 and z-CNN 2x2/s2 (compile-time windows), odd extents (clamped taps),
    # and windows that take the generic runtime-k loops (3x3/s1 backward, 5x5)
    for (N, H, W, C, k, s, p) in [(2, 16, 16, 64, 3, 2, 1), (2, 14, 14, 32, 2, 2, 0), (1, 15, 13, 64, 3, 2, 1),
                                  (1, 9, 9, 32, 3, 1, 1), (1, 11, 11, 32, 5, 2, 2)]:
        x = torch.randn(N, C, H, W, generator=g)
        x = F.relu(x)                         # many exact ties (zeros), as after ReLU
        if dtype == torch.bfloat16:
            x = x.bfloat16().float()
        Ho, Wo = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
        xd = _nhwc(x).to(dev, dtype)
        y = torch.empty(N, Ho, Wo, C, device=dev, dtype=dtype)
        am = torch.empty(N, Ho, Wo, C, device=dev, dtype=torch.uint8)
        call("maxpool_fwd", dt, xd, y, am, N, H, W, C, k, s, p, Ho, Wo, stream())
        xr = x.clone().requires_grad_(True)
        yr = F.max_pool2d(xr, k, s, p)
        assert torch.equal(y.float().cpu().permute(0, 3, 1, 2), yr.detach())
        dy = torch.randn(N, C, Ho, Wo, generator=g)
        if dtype == torch.bfloat16:
            dy = dy.bfloat16().float()
        yr.backward(dy)
        dx = torch.empty_like(xd)
        call("maxpool_bwd", dt, _nhwc(dy).to(dev, dtype), am, dx, N, H, W, C, k, s, p, Ho, Wo, stream())
        _close(dx.permute(0, 3, 1, 2), xr.grad, 1e-6 if dtype == torch.float32 else 1e-2, "maxpool bwd")
        # BN-apply + ReLU + pool in one pass == bn_act_fwd then maxpool_fwd, bit for bit
        yraw = _nhwc(torch.randn(N, C, H, W, generator=g)).to(dev, dtype)
        sc = (torch.rand(C, generator=g) + 0.5).to(dev)
        sh = (torch.randn(C, generator=g) * 0.5).to(dev)
        act = torch.empty_like(yraw)
        call("bn_act_fwd", dt, yraw, sc, sh, None, None, None, 1, act, N * H * W, C, stream())
        y1, a1 = torch.empty_like(y), torch.empty_like(am)
        call("maxpool_fwd", dt, act, y1, a1, N, H, W, C, k, s, p, Ho, Wo, stream())
        y2, a2 = torch.empty_like(y), torch.empty_like(am)
        call("bn_relu_maxpool_fwd", dt, yraw, sc, sh, y2, a2, N, H, W, C, k, s, p, Ho, Wo, stream())
        torch.cuda.synchronize()
        assert torch.equal(y1, y2) and torch.equal(a1, a2)
    x = torch.randn(2, 64, 7, 7, generator=g)
    f = torch.empty(2, 64, device=dev)
    call("avgpool_fwd", 0, _nhwc(x).to(dev), f, 2, 49, 64, stream())
    _close(f, x.mean((2, 3)), 1e-6, "avgpool")


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("O,I,k,cpad,stride", [(64, 3, 7, 4, 1), (64, 3, 7, 4, 2), (32, 3, 7, 4, 2),
                                                (256, 64, 1, 64, 1), (64, 64, 3, 64, 1), (512, 512, 3, 512, 1),
                                                (2048, 1024, 1, 1024, 1), (100, 72, 3, 72, 2)])
def test_pack_layouts(dtype, O, I, k, cpad, stride):
    """pose6d_pack_conv_weights: wp[o][(kh, kw', ci)] with channel / K zero padding --
    kw' = kw, or for the 4-channel stride-2 7x7 stems (pose6d_conv_pack_geom) the
    row-tap layout, 8 taps per kernel row with a zero tap in front -- and
    wt[ci][kh][kw][o], exactly the dtype-rounded OIHW values."""
    from pose6d.trunk import pack_geom, pack_single
    g = torch.Generator(device="cuda").manual_seed(O + I + k)
    w = torch.randn(O, I, k, k, device="cuda", generator=g)
    wp, wt = pack_single(w, cpad, dtype, with_t=I >= 8, stride=stride)
    torch.cuda.synchronize()
    kwp, _ = pack_geom(dtype, cpad, k, stride, k // 2)
    assert kwp == (8 if (cpad == 4 and stride == 2 and k == 7) else k)
    ref = torch.zeros(O, k, kwp, cpad, device="cuda")
    ref[:, :, kwp - k:, :I] = w.permute(0, 2, 3, 1)
    ref = ref.reshape(O, -1)
    Kpad = wp.shape[1]
    full = torch.zeros(O, Kpad, device="cuda")
    full[:, :ref.shape[1]] = ref
    assert torch.equal(wp.float(), full.to(dtype).float())
    if I >= 8:
        assert torch.equal(wt.float(), w.permute(1, 2, 3, 0).to(dtype).float())


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("N,C,H,W,Cp", [(2, 3, 224, 224, 4), (3, 3, 7, 5, 4), (1, 4, 8, 8, 4), (2, 3, 6, 6, 8)])
def test_nchw_to_nhwc(dtype, N, C, H, W, Cp):
    """The model-input conversion (vectorised 4-pixel form when H*W % 4 == 0 and Cpad ==
    4, per-element otherwise) equals torch's permute + zero channel padding exactly."""
    from pose6d._lib import call, stream
    from pose6d.trunk import DTYPES
    x = torch.randn(N, C, H, W, generator=torch.Generator().manual_seed(3)).cuda()
    y = torch.full((N, H, W, Cp), 7.0, device="cuda", dtype=dtype)
    call("nchw_to_nhwc", DTYPES[dtype], x, y, N, C, H, W, Cp, stream())
    ref = torch.zeros(N, H, W, Cp, dtype=dtype)
    ref[..., :C] = x.cpu().permute(0, 2, 3, 1).to(dtype)
    torch.cuda.synchronize()
    assert torch.equal(y.cpu(), ref)
