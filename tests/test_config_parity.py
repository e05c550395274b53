"""Parity at BASELINE.json's own configuration sizes (the benchmarked paths).

* configs[1]: PoseNetRGB, batch 32, 224^2, fp32 -- the drop-in module's eval
  forward against the oracle's torch-CPU fp32 restatement, 1e-4 relative.
* configs[2]: RGBDGeometricTrainer at batch 32 (forward + PoseLoss(1, 10) +
  backward + clip_grad_norm_(1.0) + AdamW, train_rgbd_geometric.py:97-115),
  replayed from its hipGraph as bench.py runs it:
  - fp32 trainer end to end against the fp32 oracle (judged against an fp64 run of
    the oracle, as tests/test_models.py does) plus the fused clip + AdamW update
    against torch's clip_grad_norm_ + AdamW on the same gradients;
  - the benchmarked bf16 trainer op by op ("teacher forced"): every conv forward,
    BN statistics + apply, pooling, the fp32 head + loss, every BN backward, every
    conv weight gradient, every data gradient (the 16 residual junctions as the sum
    of their consumers' contributions) and the stem's max-pool backward are checked
    against torch-CPU fp32 ops applied to the SAME bf16 operands the step used.
    End-to-end fp32-vs-bf16 comparison is meaningless for a random-init ResNet50:
    on the oracle itself, rounding only the input image to bf16 (0.4 %) moves
    the pooled features by 4.7 % and the head output by 43 % (BN1d over 32
    near-identical feature vectors amplifies it; tools/diag_config_parity.py).
    Tolerances: stored bf16 tensors within one bf16 ulp (2^-7 relative; rounding
    alone is <= 2^-8, accumulation order can move a value across a rounding
    boundary) + 1e-3 of the tensor's RMS; fp32
    sums of bf16 products (weight gradients, BN affine gradients) within 1e-3
    relative (Frobenius); BN statistics within 1e-3.
Dropout modules are in eval (their RNG differs from torch's by construction)."""
import warnings

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from oracle import pose_loss as OP
from oracle import resnet as OR


def _rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return ((a - b).abs().max() / (b.abs().max() + 1e-30)).item()


def _frob(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return ((a - b).norm() / (b.norm() + 1e-300)).item()


@pytest.mark.gpu
def test_configs1_posenet_rgb_bs32_fp32_eval():
    from models.pose_net_rgb import PoseNetRGB
    warnings.simplefilter("ignore")
    torch.manual_seed(0)
    m = PoseNetRGB(pretrained=False)
    P = {k: v.clone() for k, v in m.state_dict().items()}
    m = m.cuda().set_compute_dtype(torch.float32).eval()
    x = torch.randn(32, 3, 224, 224, generator=torch.Generator().manual_seed(31))
    with torch.no_grad():
        rot, trans = m(x.cuda())
        rr, tr = OR.forward_rgb(P, x, False)
    for got, ref, what in ((rot, rr, "rotation"), (trans, tr, "translation")):
        got = got.cpu()
        err = (got - ref).abs()
        scale = ref.abs().max().item()
        assert bool((err <= 1e-4 * ref.abs() + 1e-4 * scale).all()), f"{what}: max err {err.max():.3e}"


def _trainer(dtype, B=32, seed=2024):
    from bench import synth_batch
    from models.pose_net_rgbd_geometric import PoseNetRGBDGeometric
    from pose6d.train import RGBDGeometricTrainer
    warnings.simplefilter("ignore")
    torch.manual_seed(0)
    m = PoseNetRGBDGeometric(pretrained=False)
    P0 = {k: v.clone() for k, v in m.state_dict().items()}
    m = m.cuda()
    tr = RGBDGeometricTrainer(m, B, dtype=dtype)               # (puts the model in train mode)
    for mod in m.modules():
        if isinstance(mod, torch.nn.Dropout):
            mod.eval()
    data = synth_batch(B, torch.device("cuda"), seed=seed)
    snap = tr.snapshot()
    tr.capture(data, warmup=1)                                # the benchmarked hipGraph step ...
    tr.restore(snap)                                          # ... replayed from the initial state
    before = tr.arena.flat.clone()
    tr.step()
    torch.cuda.synchronize()
    return tr, P0, data, before


def _check_adamw(tr, before):
    """The fused clip-norm + AdamW at full size against torch on our own gradients."""
    params = [torch.nn.Parameter(before[o:o + p.numel()].view_as(p).clone())
              for p, o in zip(tr.arena.params, tr.arena.offsets)]
    for q, p, o in zip(params, tr.arena.params, tr.arena.offsets):
        q.grad = tr.arena.grad[o:o + p.numel()].view_as(p).clone()
    torch.nn.utils.clip_grad_norm_(params, 1.0)
    torch.optim.AdamW(params, lr=1e-4, weight_decay=1e-4).step()
    for q, p in zip(params, tr.arena.params):
        np.testing.assert_allclose(p.detach().cpu().numpy(), q.detach().cpu().numpy(), rtol=1e-6, atol=1e-9)


def _oracle_step(P0, data, dtype):
    cpu = [t.cpu().to(dtype) if t.is_floating_point() else t.cpu() for t in data]
    P = {k: (v.clone().to(dtype).requires_grad_(True) if v.is_floating_point() and "running" not in k
             else (v.clone().to(dtype) if v.is_floating_point() else v.clone())) for k, v in P0.items()}
    rot, trans = OR.forward_rgbd_geometric(P, cpu[0], None, cpu[1], cpu[2], cpu[3], True)
    loss = OP.pose_loss(rot, trans, cpu[4], cpu[5], 1.0, 10.0)
    loss.backward()
    return rot.detach(), trans.detach(), loss.detach(), P


@pytest.mark.gpu
def test_configs2_trainer_bs32_fp32_end_to_end():
    tr, P0, data, before = _trainer(torch.float32)
    r32, t32, L32, P32 = _oracle_step(P0, data, torch.float32)
    r64, t64, L64, P64 = _oracle_step(P0, data, torch.float64)

    def check(ours, ref32, ref64, what):
        e, e_ref = _rel(ours, ref64), _rel(ref32, ref64)
        assert e <= max(1e-4, 3 * e_ref), f"{what}: ours {e:.2e} vs exact, reference fp32 {e_ref:.2e}"

    check(tr.rot, r32, r64, "rotation")
    check(tr.trans, t32, t64, "translation")
    check(tr.loss, L32, L64, "loss")
    named = dict(tr.model.named_parameters())
    ours, ref = [], []
    for k, v in P64.items():
        if isinstance(v, torch.Tensor) and v.grad is not None:
            ours.append(_frob(tr.arena.grad_of(named[k]), v.grad))
            ref.append(_frob(P32[k].grad, v.grad))
    ours, ref = np.array(ours), np.array(ref)
    assert np.median(ours) <= 2 * np.median(ref) + 1e-5, (np.median(ours), np.median(ref))
    assert ours.max() <= 3 * ref.max() + 1e-5, (ours.max(), ref.max())
    sd = tr.model.state_dict()
    for k in P0:
        if "running" in k:
            check(sd[k], P32[k], P64[k], k)
        elif "num_batches" in k:
            assert int(sd[k]) == int(P32[k]), k
    _check_adamw(tr, before)


def _nchw(t):
    return t.detach().permute(0, 3, 1, 2).float().cpu()


class _Tol:
    """Collects (error / tolerance) per check; asserts all <= 1 at the end."""

    def __init__(self):
        self.worst = {}

    def stored(self, what, got, ref, extra=None):
        # a bf16 tensor that should be bf16(ref): one bf16 ulp + 1e-3 of the RMS (+ `extra`:
        # an elementwise allowance for intermediates rounded to bf16 inside the kernel)
        got, ref = got.double(), ref.double()
        rms = ref.pow(2).mean().sqrt().item() + 1e-30
        tol = 2.0 ** -7 * ref.abs() + 1e-3 * rms
        if extra is not None:
            tol = tol + extra.double()
        r = ((got - ref).abs() / tol).max().item()
        self._put(what, r)

    def sums(self, what, got, ref, tol=1e-3):
        self._put(what, _frob(got, ref) / tol)

    def _put(self, what, r):
        kind = what.split(":")[0]
        if r > self.worst.get(kind, (0, ""))[0]:
            self.worst[kind] = (r, what)

    def check(self):
        print({k: (round(v[0], 3), v[1]) for k, v in self.worst.items()})
        bad = {k: v for k, v in self.worst.items() if v[0] > 1.0}
        assert not bad, bad


def _check_pool_bwd(T, pool):
    """The stem's max-pool backward: the pooled gradient routed to the input pixel the
    forward's argmax names (window index kh * k + kw; the first maximum), summed over the
    windows that share a pixel.  The argmax is checked too: the pixel it names must hold
    the window's maximum of the reference pool input (within the stored tolerance)."""
    a, c = pool.act, pool.act.cop
    B, Ho, Wo, C = pool.argmax.shape
    H, W, k, s, p = pool.src.H, pool.src.W, pool.k, pool.s, pool.p
    idx = pool.argmax.long().cpu()
    oy = torch.arange(Ho).view(1, Ho, 1, 1)
    ox = torch.arange(Wo).view(1, 1, Wo, 1)
    iy, ix = oy * s - p + idx // k, ox * s - p + idx % k
    assert bool(((iy >= 0) & (iy < H) & (ix >= 0) & (ix < W)).all()), "argmax names a padding position"
    n = torch.arange(B).view(B, 1, 1, 1)
    ch = torch.arange(C).view(1, 1, 1, C)
    flat = (((n * H + iy) * W + ix) * C + ch).flatten()
    dy = pool.out.g.detach().float().cpu().flatten()
    ref = torch.zeros(B * H * W * C).index_add_(0, flat, dy).view(B, H, W, C).permute(0, 3, 1, 2)
    T.stored(f"pool bwd:{a.out.name}", _nchw(a.out.g), ref)
    # the pool input the kernel saw: bf16(max(y * scale + shift, 0))
    y = c.out.t.detach().double().cpu()
    z = (y * c.scale.cpu().double() + c.shift.cpu().double()).clamp_min(0).float().bfloat16().float()
    picked = z.flatten()[flat].view(B, Ho, Wo, C).permute(0, 3, 1, 2)
    T.stored(f"pool argmax:{pool.out.name}", picked, _nchw(pool.out.t))


@pytest.mark.gpu
def test_configs2_trainer_bs32_bf16_teacher_forced():
    from pose6d.trunk import _ActOp, _ConvOp, _PoolOp
    tr, P0, data, before = _trainer(torch.bfloat16)
    named = dict(tr.model.named_parameters())
    pidx = {id(p): i for i, p in enumerate(tr.arena.params)}

    def w0(p):   # the parameter as the step used it (before the AdamW update)
        i = pidx[id(p)]
        o = tr.arena.offsets[i]
        return before[o:o + p.numel()].view_as(p).detach().cpu().float()

    def grad(p):
        return tr.arena.grad_of(p).detach().cpu().float()

    T = _Tol()
    trunk = tr.trunk
    for op in trunk.ops:
        if isinstance(op, _ConvOp):
            x = _nchw(op.src.t)[:, :op.cin]
            Wb = w0(op.conv.weight).bfloat16().float()
            y = F.conv2d(x, Wb, None, op.stride, op.pad)
            T.stored(f"conv fwd:{op.out.name}", _nchw(op.out.t), y)
            # batch statistics of the fp32 accumulators
            mu = y.mean(dim=(0, 2, 3))
            var = y.var(dim=(0, 2, 3), unbiased=False)
            inv = (var + op.bn.eps).rsqrt()
            T._put(f"bn stats:{op.out.name}", ((op.mean.cpu() - mu).abs() / (var.sqrt() + 1e-12)).max().item() / 1e-3)
            T.sums(f"bn stats:{op.out.name}.inv", op.inv.cpu(), inv)
        elif isinstance(op, _ActOp):
            c = op.cop
            z = _nchw(c.out.t) * c.scale.cpu().view(1, -1, 1, 1) + c.shift.cpu().view(1, -1, 1, 1)
            if op.res_conv is not None:
                r = op.res_conv
                z = z + (_nchw(r.out.t) * r.scale.cpu().view(1, -1, 1, 1) + r.shift.cpu().view(1, -1, 1, 1))
            elif op.res_act is not None:
                z = z + _nchw(op.res_act.t)
            if op.relu:
                z = z.clamp_min(0)
            op._ref_out = z
            if not op.pooled:
                T.stored(f"bn act:{op.out.name}", _nchw(op.out.t), z)
        elif isinstance(op, _PoolOp):
            src = op.act._ref_out.bfloat16().float() if op.act is not None else _nchw(op.src.t)
            T.stored(f"pool:{op.out.name}", _nchw(op.out.t), F.max_pool2d(src, op.k, op.s, op.p))
    f = trunk.final
    feat = trunk.feat.detach().cpu()
    T.sums("avgpool:feat", feat, _nchw(f.t).mean(dim=(2, 3)), 1e-5)

    # fp32 head + normalise + loss + their backward, from our own features
    P = {k: (w0(named[k]).clone().requires_grad_(True) if k in named else v.clone())
         for k, v in P0.items() if k.startswith("rot_head")}
    fx = feat.clone().requires_grad_(True)
    rot = OR.normalize(OR.bn_mlp(fx, P, "rot_head", [2048, 1024, 512, 4], True))
    cpu = [t.cpu() for t in data]
    trans = OR.pinhole_rgbd_geometric(cpu[1], cpu[2], cpu[3])
    loss = OP.pose_loss(rot, trans, cpu[4], cpu[5], 1.0, 10.0)
    loss.backward()
    T.sums("head:rot", tr.rot.cpu(), rot.detach(), 1e-4)
    T.sums("head:loss", tr.loss.cpu().view(1), loss.detach().view(1), 1e-5)
    assert torch.equal(tr.trans.cpu(), trans)
    T.sums("head:dfeat", tr.head.stages[0].dx.cpu(), fx.grad, 1e-4)
    for k, v in P.items():
        if v.grad is None:
            continue
        if k in ("rot_head.0.bias", "rot_head.4.bias"):
            # a Linear bias feeding BatchNorm1d: its gradient is 0 analytically (the batch
            # mean is removed); both sides are rounding noise -> judged against the weight's
            w = grad(named[k[:-4] + "weight"]).abs().max().item()
            T._put(f"head:grad {k}", (grad(named[k]) - v.grad).abs().max().item() / (1e-4 * w))
        else:
            T.sums(f"head:grad {k}", grad(named[k]), v.grad, 1e-4)

    # backward: BN (from our dout), conv weight gradients, and every data gradient where
    # the contributions meet -- a conv input's gradient is the sum over its consumers:
    # each reading conv's data gradient, plus, for a block input, the identity branch's
    # share dout * mask of the block output (added in the conv1 data-gradient epilogue),
    # or the downsample conv's data gradient (added in place after conv1's)
    for op in trunk.ops:
        if isinstance(op, _ActOp):
            c = op.cop
            dout = _nchw(op.out.g)
            y = _nchw(c.out.t)
            if op.pooled:
                # the stem: its BN + ReLU lives in the max pool; the backward recomputes the
                # ReLU sign from y (exact in fp64: fmaf rounding keeps the sign)
                pre = y.double() * c.scale.cpu().double().view(1, -1, 1, 1) + c.shift.cpu().double().view(1, -1, 1, 1)
                mask = (pre > 0).float()
            else:
                # the ReLU mask the kernels use: stored output > 0
                mask = (_nchw(op.out.t) > 0).float() if op.relu else torch.ones_like(y)
            dz = dout * mask
            xh = (y - c.mean.cpu().view(1, -1, 1, 1)) * c.inv.cpu().view(1, -1, 1, 1)
            M = y.numel() // y.shape[1]
            s1, s2 = dz.sum(dim=(0, 2, 3)), (dz * xh).sum(dim=(0, 2, 3))
            g = w0(c.bn.weight)
            dy = (g * c.inv.cpu()).view(1, -1, 1, 1) * (dz - (s1 / M).view(1, -1, 1, 1) - xh * (s2 / M).view(1, -1, 1, 1))
            T.stored(f"bn bwd:{op.out.name}", _nchw(c.out.g), dy)
            T.sums(f"bn grad:{op.out.name}.beta", grad(c.bn.bias), s1)
            T.sums(f"bn grad:{op.out.name}.gamma", grad(c.bn.weight), s2)
        elif isinstance(op, _ConvOp):
            x = _nchw(op.src.t)[:, :op.cin]
            Wb = w0(op.conv.weight).bfloat16().float()
            dy = _nchw(op.out.g)
            dW = torch.nn.grad.conv2d_weight(x, Wb.shape, dy, op.stride, op.pad)
            T.sums(f"conv wgrad:{op.out.name}", grad(op.conv.weight), dW)
        elif isinstance(op, _PoolOp) and op.act is not None:
            _check_pool_bwd(T, op)
    contrib = {}
    for op in trunk.ops:
        if isinstance(op, _ConvOp) and op.needs_dgrad:
            x = _nchw(op.src.t)[:, :op.cin]
            Wb = w0(op.conv.weight).bfloat16().float()
            dx = torch.nn.grad.conv2d_input(x.shape, Wb, _nchw(op.out.g), op.stride, op.pad)
            contrib.setdefault(id(op.src), (op.src, []))[1].append(("conv", dx))
        elif isinstance(op, _ActOp) and op.res_act is not None:
            mask = (_nchw(op.out.t) > 0).float() if op.relu else 1.0
            contrib.setdefault(id(op.res_act), (op.res_act, []))[1].append(("res", _nchw(op.out.g) * mask))
    junctions = 0
    for src, parts in contrib.values():
        kind = "conv dgrad" if len(parts) == 1 else "junction dgrad"
        junctions += len(parts) > 1
        extra = None
        if len(parts) > 1:
            # the data-gradient epilogue rounds its accumulator to bf16 (the tile is staged
            # through LDS as T) before it adds the waiting contribution -- the identity
            # branch's dout * mask, or conv1's stored data gradient that the downsample
            # conv's epilogue accumulates in place -- exactly as a separate add of two
            # bf16 tensors would: each conv term carries one bf16 rounding of its own
            extra = 2.0 ** -7 * sum(t.abs() for k, t in parts if k == "conv")
        T.stored(f"{kind}:{src.name}", _nchw(src.g), sum(t for _, t in parts), extra)
    assert junctions == 16, junctions   # every Bottleneck's input: 4 downsampling + 12 identity blocks
    T.check()
    _check_adamw(tr, before)


@pytest.mark.gpu
def test_configs2_eval_forward_bs32_bf16_teacher_forced():
    """The north-star forward metric's path (bench.py forward_roofline_eval): the
    PoseNetRGBDGeometric eval forward at batch 32 in bf16 (model.eval(), as the
    reference's validation loop runs it, train_rgbd_geometric.py:120-136), checked op
    by op against torch-CPU fp32 ops on the SAME bf16 operands, with non-trivial
    running statistics.  Covers pose6d_bn_eval_fold (scale / shift from the running
    statistics), pose6d_conv2d_fwd_act (conv + BN + residual + ReLU in the epilogue),
    pose6d_conv2d_fwd_act_dual (a downsampling block's conv3 + downsample conv + both
    BNs in one launch), the stem conv + pose6d_bn_relu_maxpool_fwd, the average pool,
    and the head's pose6d_gemm_f32_bn_eval; tolerances as the training teacher-forced
    test above."""
    from bench import synth_batch
    from models.pose_net_rgbd_geometric import PoseNetRGBDGeometric
    from pose6d.trunk import _ActOp, _ConvOp, _PoolOp
    warnings.simplefilter("ignore")
    torch.manual_seed(0)
    m = PoseNetRGBDGeometric(pretrained=False)
    g = torch.Generator().manual_seed(77)
    for mod in m.modules():
        if isinstance(mod, (torch.nn.BatchNorm2d, torch.nn.BatchNorm1d)):
            C = mod.num_features
            mod.running_mean.copy_(torch.randn(C, generator=g) * 0.1)
            mod.running_var.copy_(torch.rand(C, generator=g) * 0.5 + 0.5)
            mod.weight.data.copy_(torch.rand(C, generator=g) + 0.5)
            mod.bias.data.copy_(torch.randn(C, generator=g) * 0.1)
    P = {k: v.clone() for k, v in m.state_dict().items()}
    m = m.cuda().set_compute_dtype(torch.bfloat16).eval()
    rgb, depth_raw, bbox, K, _, _ = synth_batch(32, torch.device("cuda"), seed=4242)
    with torch.no_grad():
        rot, trans = m(rgb, None, depth_raw, bbox, K)
    torch.cuda.synchronize()
    trunk = m.engines()["backbone"]
    dual = trunk._dual_pairs()
    assert dual, "batch 32: the layer1 / layer2 downsampling blocks run as one launch"
    T = _Tol()

    def bnp(bn):
        inv = 1.0 / torch.sqrt(bn.running_var.cpu() + bn.eps)
        sc = bn.weight.detach().cpu() * inv
        return sc, bn.bias.detach().cpu() - bn.running_mean.cpu() * sc

    def raw(op):   # conv of the stored bf16 input with the bf16 weights, rounded as stored
        x = _nchw(op.src.t)[:, :op.cin]
        return F.conv2d(x, op.conv.weight.detach().cpu().bfloat16().float(), None, op.stride,
                        op.pad).bfloat16().float()

    ref_act = {}
    for op in trunk.ops:
        if isinstance(op, _ConvOp):
            sc, sh = bnp(op.bn)
            T.sums(f"bn eval fold:{op.out.name}.scale", op.scale.cpu(), sc, 1e-6)
            T.sums(f"bn eval fold:{op.out.name}.shift", op.shift.cpu(), sh, 1e-6)
        elif isinstance(op, _ActOp):
            c = op.cop
            sc, sh = bnp(c.bn)
            y = raw(c)
            if op.pooled:
                T.stored(f"conv fwd:{c.out.name}", _nchw(c.out.t), y)   # the stem's raw output is stored
                y = _nchw(c.out.t)
            z = y * sc.view(1, -1, 1, 1) + sh.view(1, -1, 1, 1)
            # the fused epilogue rounds the conv accumulator to bf16 before the BN, as the
            # separate launches' stored output was: that rounding may land one bf16 ulp
            # away from bf16(our fp32 conv) (other summation order), scaled by the BN
            flip = 2.0 ** -7 * y.abs() * sc.abs().view(1, -1, 1, 1) if not op.pooled else None
            if op.res_conv is not None:
                r = op.res_conv
                rs, rb = bnp(r.bn)
                yr = raw(r) if c in dual else _nchw(r.out.t)
                if c not in dual:
                    T.stored(f"conv fwd:{r.out.name}", _nchw(r.out.t), raw(r))
                else:
                    flip = flip + 2.0 ** -7 * yr.abs() * rs.abs().view(1, -1, 1, 1)
                z = z + (yr * rs.view(1, -1, 1, 1) + rb.view(1, -1, 1, 1))
            elif op.res_act is not None:
                z = z + _nchw(op.res_act.t)
            if op.relu:
                z = z.clamp_min(0)
            ref_act[id(op)] = z
            if not op.pooled:
                kind = "fwd act dual" if c in dual else "fwd act"
                T.stored(f"{kind}:{op.out.name}", _nchw(op.out.t), z, flip)
        elif isinstance(op, _PoolOp):
            src = ref_act[id(op.act)].bfloat16().float() if op.act is not None else _nchw(op.src.t)
            T.stored(f"pool:{op.out.name}", _nchw(op.out.t), F.max_pool2d(src, op.k, op.s, op.p))
    feat = trunk.feat.detach().cpu()
    T.sums("avgpool:feat", feat, _nchw(trunk.final.t).mean(dim=(2, 3)), 1e-5)
    # eval head (Linear + BatchNorm1d + ReLU fused GEMMs) + normalise from our own features
    ref_rot = OR.normalize(OR.bn_mlp(feat, {k: v for k, v in P.items() if k.startswith("rot_head")}, "rot_head",
                                     [2048, 1024, 512, 4], False))
    T.sums("head:rot", rot.cpu(), ref_rot, 1e-4)
    assert torch.equal(trans.cpu(), OR.pinhole_rgbd_geometric(depth_raw.cpu(), bbox.cpu(), K.cpu()))
    T.check()
