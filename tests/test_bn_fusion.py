"""BatchNorm fusions on the residual path: the ReLU bits pose6d_bn_act_fwd_mask stores
give pose6d_bn_bwd_mask exactly what pose6d_bn_bwd computes from the forward output."""
import pytest
import torch

pytestmark = pytest.mark.gpu

@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_relu_mask_bits_match_output(dtype):
    """pose6d_bn_act_fwd_mask's bits give pose6d_bn_bwd_mask exactly what
    pose6d_bn_bwd computes from the forward output (residual BN + ReLU)."""
    from pose6d._lib import DT_BF16, DT_F32, call, stream
    dt = DT_BF16 if dtype == torch.bfloat16 else DT_F32
    E = 8 if dtype == torch.bfloat16 else 4
    M, C, dev = 2000, 256, "cuda"
    g = torch.Generator(device=dev).manual_seed(5)
    y = (torch.randn(M, C, device=dev, generator=g) * 2).to(dtype)
    res = torch.randn(M, C, device=dev, generator=g).to(dtype)
    sc = torch.rand(C, device=dev, generator=g) + 0.5
    sh = torch.randn(C, device=dev, generator=g)
    out = torch.empty_like(y)
    mb = torch.empty(M * C // E, device=dev, dtype=torch.uint8)
    call("bn_act_fwd_mask", dt, y, sc, sh, res, None, None, 1, out, mb, M, C, stream())
    bits = ((mb.long()[:, None] >> torch.arange(E, device=dev)) & 1).reshape(M, C)
    assert torch.equal(bits.bool(), out.float() > 0)
    dout = torch.randn(M, C, device=dev, generator=g).to(dtype)
    mean, inv, gam = torch.randn(C, device=dev, generator=g), torch.rand(C, device=dev, generator=g) + .5, sc
    from pose6d._lib import query
    ws = torch.empty((query("bn_bwd_workspace_rows", M) * 2 + 3) * C, device=dev)
    outs = []
    for use_bits in (False, True):
        dy, dz = torch.empty_like(y), torch.empty_like(y)
        dg, db = torch.empty(C, device=dev), torch.empty(C, device=dev)
        if use_bits:
            call("bn_bwd_mask", dt, dout, mb, y, mean, inv, gam, dg, db, 0, dy, dz, ws, M, C, stream())
        else:
            call("bn_bwd", dt, dout, out, None, None, y, mean, inv, gam, dg, db, 0, dy, dz, ws, M, C, stream())
        outs.append((dy, dz, dg, db))
    torch.cuda.synchronize()
    for a, b in zip(*outs):
        assert torch.equal(a, b)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("M,C", [(2000, 256), (12544, 2048), (37, 64)])
@pytest.mark.parametrize("acc", [0, 1])
def test_dual_bn_backward_matches_two_calls(dtype, M, C, acc):
    """pose6d_bn_bwd_mask_dual (a downsampling block's last BN + branch BN, one dout and
    one mask) = pose6d_bn_bwd_mask on each, bit for bit, written and accumulated, with a
    ragged row count."""
    from pose6d._lib import DT_BF16, DT_F32, call, query, stream
    dt = DT_BF16 if dtype == torch.bfloat16 else DT_F32
    E = 8 if dtype == torch.bfloat16 else 4
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(M + C)
    r = lambda *s: torch.randn(*s, device=dev, generator=g)
    dout = r(M, C).to(dtype)
    mb = torch.randint(0, 256, (M * C // E,), device=dev, dtype=torch.uint8, generator=g)
    bns = []
    for _ in range(2):
        bns.append(((r(M, C) * 2).to(dtype), r(C), torch.rand(C, device=dev, generator=g) + .5,
                    torch.rand(C, device=dev, generator=g) + .5))
    one = (query("bn_bwd_workspace_rows", M) * 2 + 3) * C
    ws = torch.empty(2 * one, device=dev)
    init = [(r(C), r(C)) for _ in range(2)]
    sep, dual = [], []
    for (y, mean, inv, gam), (g0, b0) in zip(bns, init):
        dy, dg, db = torch.empty_like(y), g0.clone(), b0.clone()
        call("bn_bwd_mask", dt, dout, mb, y, mean, inv, gam, dg, db, acc, dy, None, ws, M, C, stream())
        sep.append((dy, dg, db))
    outs = [(torch.empty_like(b[0]), i[0].clone(), i[1].clone()) for b, i in zip(bns, init)]
    (y, mean, inv, gam), (y2, mean2, inv2, gam2) = bns
    (dy, dg, db), (dy2, dg2, db2) = outs
    call("bn_bwd_mask_dual", dt, dout, mb, y, mean, inv, gam, dg, db, dy, y2, mean2, inv2, gam2, dg2, db2, dy2, acc,
         ws, M, C, stream())
    torch.cuda.synchronize()
    for a, b in zip(sep, outs):
        for u, v in zip(a, b):
            assert torch.equal(u, v)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_trunk_backward_dual_bn_is_bit_identical(dtype):
    """Training trunk backward with the dual BN backward in the four downsampling blocks
    equals the two-call path bit for bit (every parameter gradient)."""
    from pose6d.resnet import resnet50_trunk
    from pose6d.trunk import TrunkEngine
    torch.manual_seed(0)
    seq = resnet50_trunk(3).cuda().train()
    eng = TrunkEngine(seq, 3)
    eng.set_dtype(dtype)
    g = torch.Generator().manual_seed(3)
    x = torch.randn(4, 3, 96, 96, generator=g).cuda()
    dfeat = torch.randn(4, 2048, generator=g).cuda()
    grads = []
    for dual in (False, True):
        eng.bwd_dual_bn = dual
        gd = {p: torch.zeros_like(p, dtype=torch.float32) for p in seq.parameters()}
        eng.forward(x, True)
        eng.backward(dfeat, lambda p: gd[p])
        torch.cuda.synchronize()
        grads.append(gd)
    assert sum(1 for op in eng.ops if getattr(op, "res_conv", None) is not None) == 4
    for p in seq.parameters():
        assert torch.equal(grads[0][p], grads[1][p])


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_trunk_forward_dual_bn_finalize_is_bit_identical(dtype):
    """Training trunk forward with each downsampling block's bn3 + downsample-BN
    finalize as ONE launch (pose6d_bn_finalize_dual) equals the two-call path bit for
    bit: features, running statistics, num_batches_tracked, saved mean / invstd."""
    from pose6d.resnet import resnet50_trunk
    from pose6d.trunk import TrunkEngine
    torch.manual_seed(0)
    seq = resnet50_trunk(3).cuda().train()
    eng = TrunkEngine(seq, 3)
    eng.set_dtype(dtype)
    g = torch.Generator().manual_seed(7)
    x = torch.randn(4, 3, 96, 96, generator=g).cuda()
    init = {k: v.clone() for k, v in seq.state_dict().items()}
    res = []
    for dual in (False, True):
        seq.load_state_dict(init)
        eng.bn_dual_finalize = dual
        feat = eng.forward(x, True).clone()
        saved = [t.clone() for op in eng.convs for t in (op.mean, op.inv, op.scale, op.shift)]
        torch.cuda.synchronize()
        res.append((feat, {k: v.clone() for k, v in seq.state_dict().items()}, saved))
    assert torch.equal(res[0][0], res[1][0])
    for k in init:
        assert torch.equal(res[0][1][k], res[1][1][k]), k
    assert int(res[1][1]["4.0.downsample.1.num_batches_tracked"]) == 1
    for a, b in zip(res[0][2], res[1][2]):
        assert torch.equal(a, b)


def _nhwc(t):
    return t.permute(0, 2, 3, 1).contiguous()


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("cfg", [(4, 14, 14, 256, 64, 1, 1, 0), (2, 14, 14, 64, 64, 3, 1, 1),
                                 (2, 28, 28, 128, 128, 3, 2, 1), (3, 7, 7, 512, 2048, 1, 1, 0)])
@pytest.mark.parametrize("kind", ["plain", "mask", "mask_res", "dual"])
def test_backward_bn_reduce_partials(cfg, dtype, kind):
    """pose6d_conv2d_backward_chain_bn: dX bit-identical to the chain without the BN
    reduce; its per-tile partials sum (float64 over rows) to sum(dz) and sum(dz * xhat)
    of that dX within fp32 summation error; pose6d_bn_bwd_partials then gives the
    three-pass backward's dy / dgamma / dbeta within one rounding of the dy type."""
    import ctypes
    from pose6d._lib import DT_BF16, DT_F32, call, query, stream
    from pose6d.trunk import _BnReduce, _WgradReduce, pack_single
    N, H, W, Cin, Cout, k, s, p = cfg
    dt = DT_BF16 if dtype == torch.bfloat16 else DT_F32
    E = 8 if dtype == torch.bfloat16 else 4
    g = torch.Generator().manual_seed(sum(cfg))
    dev = "cuda"
    Ho, Wo = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
    M = N * H * W
    rnd = lambda *sh: torch.randn(*sh, generator=g)
    x = _nhwc(rnd(N, Cin, H, W)).to(dev, dtype)
    _, wt = pack_single((rnd(Cout, Cin, k, k) * 0.05).to(dev), Cin, dtype)
    dy = _nhwc(rnd(N, Cout, Ho, Wo)).to(dev, dtype)
    # the BN(s) producing this conv's input: y (pre-BN), mean, invstd, gamma, relu
    bns = [(_nhwc(rnd(N, Cin, H, W) * 2).to(dev, dtype), (rnd(Cin) * 0.3).to(dev),
            (torch.rand(Cin, generator=g) + 0.5).to(dev), (torch.rand(Cin, generator=g) + 0.5).to(dev))
           for _ in range(2)]
    sc, sh = (torch.rand(Cin, generator=g) + 0.5).to(dev), rnd(Cin).to(dev)
    bits = torch.randint(0, 256, (M * Cin // E,), generator=g, dtype=torch.uint8).to(dev)
    dres = _nhwc(rnd(N, Cin, H, W)).to(dev, dtype) if kind == "mask_res" else None
    dmask = torch.randint(0, 256, (M * Cin // E,), generator=g, dtype=torch.uint8).to(dev) if dres is not None else None
    ws = torch.empty(query("conv2d_wgrad_workspace", dt, N, Ho, Wo, Cin, Cout, k, k) // 4 + 1, device=dev)
    rows = query("conv2d_backward_bn_rows", dt, N, H, W, Cin, Cout, k, k, s, p, Ho, Wo)
    assert rows > 0
    part = torch.full((2, Cin, rows), float("nan"), device=dev)
    part2 = torch.full((2, Cin, rows), float("nan"), device=dev)
    (y, mean, inv, gam), (y2, mean2, inv2, gam2) = bns
    plain, dual = kind == "plain", kind == "dual"
    desc = _BnReduce(y.data_ptr(), mean.data_ptr(), inv.data_ptr(), sc.data_ptr() if plain else None,
                     sh.data_ptr() if plain else None, None if plain else bits.data_ptr(), part.data_ptr(),
                     y2.data_ptr() if dual else None, mean2.data_ptr() if dual else None,
                     inv2.data_ptr() if dual else None, part2.data_ptr() if dual else None, rows)
    dxs = []
    for with_bn in (False, True):
        dx = torch.full_like(x, float("nan"))
        dw = torch.empty(Cout, Cin, k, k, device=dev)
        deferred = ctypes.c_int32(0)
        tail = (dx, dw, 0, ws, ws.numel() * 4, N, H, W, Cin, Cin, Cout, k, k, s, p, Ho, Wo, None,
                ctypes.addressof(deferred))
        if with_bn:
            call("conv2d_backward_chain_bn", dt, x, dy, wt, dres, dmask, *tail, ctypes.addressof(desc), stream())
        elif dmask is not None:
            call("conv2d_backward_chain_masked", dt, x, dy, wt, dres, dmask, *tail, stream())
        else:
            call("conv2d_backward_chain", dt, x, dy, wt, dres, *tail, stream())
        if deferred.value:
            job = _WgradReduce(ws.data_ptr(), dw.data_ptr(), dt, N, H, W, Cin, Cin, Cout, k, k, s, p, Ho, Wo, 0)
            call("wgrad_reduce", ctypes.addressof(job), stream())
        torch.cuda.synchronize()
        dxs.append(dx.clone())
    assert torch.equal(dxs[0], dxs[1]), "the BN-reduce epilogue changed dX"
    dx = dxs[1].reshape(M, Cin).double()
    if plain:
        relu = ((y.float() * sc + sh).to(dtype).float() > 0).reshape(M, Cin)   # fmaf then T rounding, as the kernel
    else:
        relu = (((bits.long()[:, None] >> torch.arange(E, device=dev)) & 1).reshape(M, Cin)) > 0
    dz = torch.where(relu, dx, torch.zeros_like(dx))
    for (yy, mu, iv, _), pt in [(bns[0], part)] + ([(bns[1], part2)] if dual else []):
        xh = (yy.reshape(M, Cin).double() - mu.double()) * iv.double()
        got = pt.double().sum(-1)
        ref = torch.stack([dz.sum(0), (dz * xh).sum(0)])
        mag = torch.stack([dz.abs().sum(0), (dz * xh).abs().sum(0)])
        assert bool(((got - ref).abs() <= 1e-5 * mag + 1e-6).all()), f"partials off: {(got - ref).abs().max()}"
    # finish: partials path vs the three-pass backward on the same dout
    coef = torch.empty(6 * Cin, device=dev)
    wsb = torch.empty(2 * (query("bn_bwd_workspace_rows", M) * 2 + 3) * Cin, device=dev)
    outs = []
    for fused in (False, True):
        o = [torch.empty_like(y), torch.zeros(Cin, device=dev), torch.zeros(Cin, device=dev),
             torch.empty_like(y), torch.zeros(Cin, device=dev), torch.zeros(Cin, device=dev)]
        d = dxs[1]
        if fused:
            call("bn_bwd_partials", dt, part, rows, d, None if plain else bits, sc if plain else None,
                 sh if plain else None, y, mean, inv, gam, o[1], o[2], o[0], part2 if dual else None,
                 y2 if dual else None, mean2 if dual else None, inv2 if dual else None, gam2 if dual else None,
                 o[4], o[5], o[3] if dual else None, 0, coef, M, Cin, stream())
        elif dual:
            call("bn_bwd_mask_dual", dt, d, bits, y, mean, inv, gam, o[1], o[2], o[0], y2, mean2, inv2, gam2, o[4],
                 o[5], o[3], 0, wsb, M, Cin, stream())
        elif plain:
            call("bn_bwd", dt, d, None, sc, sh, y, mean, inv, gam, o[1], o[2], 0, o[0], None, wsb, M, Cin, stream())
        else:
            call("bn_bwd_mask", dt, d, bits, y, mean, inv, gam, o[1], o[2], 0, o[0], None, wsb, M, Cin, stream())
        torch.cuda.synchronize()
        outs.append(o)
    n = 6 if dual else 3
    for i in range(n):
        a, b = outs[0][i].float(), outs[1][i].float()
        # dy: one rounding of the dy type on the coefficient difference (fp32 sums in
        # another order); dgamma / dbeta: fp32 sums of the same terms in another order
        tol = (2.0 ** -7 if dtype == torch.bfloat16 else 1e-5) if i % 3 == 0 else 1e-5
        scale = b.abs().max().item() + 1e-12
        assert bool(((a - b).abs() <= tol * b.abs() + tol * 1e-2 * scale + 1e-7).all()), \
            f"output {i}: max diff {(a - b).abs().max().item():.3e} (scale {scale:.3e})"


def test_trunk_backward_conv_bn_reduce():
    """Training trunk backward with the BN reduce folded into the data gradients: in
    fp32 every parameter gradient equals the three-pass BN backward's within fp32
    re-association (1e-4); in bf16 the two paths round differently (the folded sums run
    in another order, so a few dy elements round the other way and that spreads through
    the 50 layers), so each is held against the fp32 gradients and the folded path must
    be as close to them as the three-pass one.  44 BNs fold (32 in-block + 12 block
    outputs feeding identity blocks)."""
    from pose6d.resnet import resnet50_trunk
    from pose6d.trunk import TrunkEngine
    torch.manual_seed(0)
    seq = resnet50_trunk(3).cuda().train()
    eng = TrunkEngine(seq, 3)
    g = torch.Generator().manual_seed(4)
    x = torch.randn(4, 3, 96, 96, generator=g).cuda()
    dfeat = torch.randn(4, 2048, generator=g).cuda()

    def grads(dtype, fold):
        eng.set_dtype(dtype)
        eng.bwd_conv_bn_reduce = fold
        gd = {p: torch.zeros_like(p, dtype=torch.float32) for p in seq.parameters()}
        eng.forward(x, True)
        eng.backward(dfeat, lambda p: gd[p])
        torch.cuda.synchronize()
        return gd

    ref = grads(torch.float32, False)
    f32 = grads(torch.float32, True)
    assert sum(1 for op in eng.ops if getattr(op, "bnr", None) is not None) == 44
    rel = lambda a, b: ((a - b).norm() / (b.norm() + 1e-20)).item()
    worst = max(rel(f32[p], ref[p]) for p in seq.parameters())
    assert worst < 1e-4, worst
    e_unf = sorted(rel(v, ref[p]) for p, v in grads(torch.bfloat16, False).items())
    e_fold = sorted(rel(v, ref[p]) for p, v in grads(torch.bfloat16, True).items())
    med = lambda e: e[len(e) // 2]
    assert med(e_fold) <= 1.25 * med(e_unf) + 1e-3, (med(e_fold), med(e_unf))
    assert e_fold[-1] <= 1.5 * e_unf[-1] + 1e-2, (e_fold[-1], e_unf[-1])


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_trunk_finalize_act_one_launch_is_bit_identical(dtype):
    """pose6d_bn_finalize_act (the training BN finalize + apply as one launch, the apply
    workgroups waiting on the finalize workgroups' ready flags) against the two launches
    it replaces (pose6d_bn_finalize + pose6d_bn_act_fwd_mask): every activation, ReLU
    mask, batch statistic, running statistic and the features bit for bit, over three
    training forwards (epochs advance), at batch 8 (rows <= 512: the one-wave fold) and
    batch 32 (layer1/2: rows > 512, the workgroup fold)."""
    import copy
    from models.pose_net_rgbd_geometric import PoseNetRGBDGeometric
    from pose6d.trunk import TrunkEngine, _ActOp, _ConvOp
    torch.manual_seed(0)
    m0 = PoseNetRGBDGeometric(pretrained=False).train()
    engs = []
    for fused in (True, False):
        m = copy.deepcopy(m0).cuda()
        e = TrunkEngine(m.backbone, 3)
        e.set_dtype(dtype)
        e.bn_fused_finalize_act = fused
        engs.append((m, e))
    for B in (8, 32):
        for it in range(3):
            x = torch.randn(B, 3, 64 if B == 32 else 96, 64 if B == 32 else 96,
                            generator=torch.Generator().manual_seed(10 * B + it)).cuda()
            feats = [e.forward(x, True).clone() for _, e in engs]
            torch.cuda.synchronize()
            assert torch.equal(feats[0], feats[1]), (B, it)
            a, b = engs[0][1], engs[1][1]
            assert sum(op.fin_flags is not None for op in a.ops if isinstance(op, _ActOp)) >= 40
            for oa, ob in zip(a.ops, b.ops):
                if not (isinstance(oa, _ActOp) and oa.pooled):   # (a pooled activation is never stored)
                    assert torch.equal(oa.out.t, ob.out.t), oa.out.name
                if isinstance(oa, _ActOp) and oa.mbits is not None:
                    assert torch.equal(oa.mbits, ob.mbits), oa.out.name
                if isinstance(oa, _ConvOp):
                    for f in ("scale", "shift", "mean", "inv"):
                        assert torch.equal(getattr(oa, f), getattr(ob, f)), (oa.out.name, f)
            for (ka, va), (kb, vb) in zip(engs[0][0].state_dict().items(), engs[1][0].state_dict().items()):
                assert torch.equal(va, vb), ka


@pytest.mark.gpu
@pytest.mark.parametrize("rows_case", ["wave_fold", "block_fold"])
def test_bn_finalize_act_fallback_is_bit_identical(rows_case):
    """The apply workgroups' own fold (taken when the finalize's ready flags do not arrive
    in time; forced here with a negative epoch) gives the finalize's scale / shift bits:
    the fused launch's outputs equal the two-launch path's."""
    import ctypes
    from pose6d._lib import DT_BF16, call, stream
    from pose6d.trunk import _BnStats
    torch.manual_seed(1)
    dev = "cuda"
    M = 6272 if rows_case == "wave_fold" else 25088   # rows 196 (<= 512) / 784
    C = 256
    rows = (M + 31) // 32
    y = (torch.randn(M, C, device=dev) * 2 + 0.3).bfloat16()
    yf = y.float()
    part = torch.zeros(2, C, rows, device=dev)
    for r in range(rows):   # the conv epilogue's (sum, M2 about the block mean) per 32 rows
        blk = yf[32 * r:32 * r + 32]
        part[0, :, r] = blk.sum(0)
        part[1, :, r] = ((blk - blk.mean(0)) ** 2).sum(0)
    res = torch.randn(M, C, device=dev).bfloat16()
    outs = []
    g0, b0 = torch.rand(C, device=dev) + 0.5, torch.randn(C, device=dev) * 0.1
    for mode in ("separate", "fallback"):
        gamma, beta = g0.clone(), b0.clone()
        rm, rv = torch.zeros(C, device=dev), torch.ones(C, device=dev)
        nbt = torch.zeros(1, device=dev, dtype=torch.int64)
        sc, sh, mu, inv = (torch.empty(C, device=dev) for _ in range(4))
        st = _BnStats(part.data_ptr(), gamma.data_ptr(), beta.data_ptr(), rm.data_ptr(), rv.data_ptr(),
                      nbt.data_ptr(), sc.data_ptr(), sh.data_ptr(), mu.data_ptr(), inv.data_ptr(), 0.1, 1e-5, C)
        out = torch.empty_like(y)
        mb = torch.empty(M * C // 8, device=dev, dtype=torch.uint8)
        if mode == "separate":
            call("bn_finalize", part, rows, C, M, gamma, beta, rm, rv, nbt, 0.1, 1e-5, 1, sc, sh, mu, inv, None,
                 stream())
            call("bn_act_fwd_mask", DT_BF16, y, sc, sh, res, None, None, 1, out, mb, M, C, stream())
        else:
            flags = torch.zeros(4096, device=dev, dtype=torch.int32)
            epoch = torch.full((1,), -5, device=dev, dtype=torch.int64)
            call("bn_finalize_act", DT_BF16, ctypes.addressof(st), rows, M, y, res, 1, out, mb, flags, epoch,
                 stream())
        torch.cuda.synchronize()
        outs.append((out, mb, sc, sh, mu, inv, rm, rv, nbt))
    for a, b in zip(*outs):
        assert torch.equal(a, b)
