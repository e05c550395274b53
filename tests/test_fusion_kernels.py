"""PoseNetRGBD fusion kernels (LayerNorm + act + dropout, cross-modal attention core)
through the C ABI, against plain torch-CPU fp32 ops fed the kernels' own dropout
masks (fp32: 1e-4 relative)."""
import pytest
import torch
import torch.nn.functional as F


def _close(got, ref, rtol, what):
    got, ref = got.detach().float().cpu(), ref.detach().float().cpu()
    scale = ref.abs().max().item() + 1e-30
    err = (got - ref).abs()
    bad = err > rtol * ref.abs() + rtol * scale
    assert not bool(bad.any()), f"{what}: max err {err.max().item():.3e} (scale {scale:.3e})"


def _act(z, act):
    return {0: z, 1: F.relu(z), 2: F.gelu(z)}[act]


@pytest.mark.gpu
@pytest.mark.parametrize("act,p", [(0, 0.0), (2, 0.0), (1, 0.3), (2, 0.2)])
def test_layernorm_fwd_bwd(act, p):
    from pose6d._lib import call, stream
    B, D, ld = 6, 1000, 1024   # strided rows on every operand (ld > D)
    g = torch.Generator().manual_seed(act * 10 + int(p * 10))
    x = torch.randn(B, ld, generator=g) * 3 + 1
    gamma, beta = torch.randn(D, generator=g), torch.randn(D, generator=g)
    dy, dy2 = torch.randn(B, ld, generator=g), torch.randn(B, ld, generator=g)
    dev = "cuda"
    xd, gd, bd = x.to(dev), gamma.to(dev), beta.to(dev)
    y = torch.zeros(B, ld, device=dev)
    y2 = torch.empty(B, D, device=dev)
    mask = torch.empty(B, D, device=dev, dtype=torch.uint8)
    mean, rstd = torch.empty(B, device=dev), torch.empty(B, device=dev)
    seed = torch.tensor([1234], dtype=torch.int64, device=dev)
    call("layernorm_fwd", xd, ld, y, ld, y2, B, D, gd, bd, 1e-5, act, p, seed, 77, mask, mean, rstd, stream())
    m = mask.cpu().float() if p > 0 else torch.ones(B, D)
    if p > 0:
        assert abs(1 - m.mean().item() - p) < 0.05
    xr = x[:, :D].clone().requires_grad_(True)
    gr, br = gamma.clone().requires_grad_(True), beta.clone().requires_grad_(True)
    yr = _act(F.layer_norm(xr, (D,), gr, br, 1e-5), act) * m / (1 - p)
    _close(y[:, :D], yr, 1e-4, "y")
    _close(y2, yr, 1e-4, "y2")
    assert torch.all(y[:, D:].cpu() == 0)   # nothing written past D
    yr.backward(dy[:, :D] + dy2[:, :D])
    dx = torch.full((B, ld), 5.0, device=dev)
    dgam, dbet = torch.full((D,), 1.0, device=dev), torch.full((D,), 2.0, device=dev)
    call("layernorm_bwd", dy.to(dev), ld, dy2.to(dev), ld, xd, ld, B, D, gd, bd, mean, rstd, act, p, mask, dx, ld, 1,
         dgam, dbet, 1, stream())
    _close(dx[:, :D] - 5.0, xr.grad, 1e-4, "dx (accumulated)")
    _close(dgam - 1.0, gr.grad, 1e-4, "dgamma (accumulated)")
    _close(dbet - 2.0, br.grad, 1e-4, "dbeta (accumulated)")


@pytest.mark.gpu
@pytest.mark.parametrize("p", [0.0, 0.1])
def test_cross_attention_core(p):
    from pose6d._lib import call, stream
    B, H, hd = 5, 8, 256
    D = H * hd
    g = torch.Generator().manual_seed(3)
    q, k, v = (torch.randn(B, D, generator=g) for _ in range(3))
    dout = torch.randn(B, D, generator=g)
    dev = "cuda"
    out = torch.empty(B, D, device=dev)
    probs = torch.empty(B, H, H, device=dev)
    mask = torch.empty(B, H, H, device=dev, dtype=torch.uint8)
    seed = torch.tensor([99], dtype=torch.int64, device=dev)
    scale = hd ** -0.5
    qd, kd, vd = q.to(dev), k.to(dev), v.to(dev)
    call("xattn_fwd", qd, kd, vd, out, B, H, hd, scale, p, seed, 5, probs, mask, stream())
    m = mask.cpu().float() if p > 0 else torch.ones(B, H, H)
    qr, kr, vr = (t.clone().requires_grad_(True) for t in (q, k, v))
    a = ((qr.view(B, H, hd) @ kr.view(B, H, hd).transpose(-2, -1)) * scale).softmax(-1)
    ref = ((a * m / (1 - p)) @ vr.view(B, H, hd)).reshape(B, D)
    _close(probs, a, 1e-5, "softmax probabilities")
    _close(out, ref, 1e-4, "attention output")
    ref.backward(dout)
    dq, dk, dv = (torch.empty(B, D, device=dev) for _ in range(3))
    call("xattn_bwd", dout.to(dev), qd, kd, vd, probs, mask, B, H, hd, scale, p, dq, dk, dv, stream())
    _close(dq, qr.grad, 1e-4, "dq")
    _close(dk, kr.grad, 1e-4, "dk")
    _close(dv, vr.grad, 1e-4, "dv")


@pytest.mark.gpu
def test_cross_modal_attention_module():
    """models.pose_net_rgbd.CrossModalAttention (engine, attention-only mode) vs the
    oracle restatement of pose_net_rgbd.py:23-35, forward and gradients."""
    import warnings
    from models.pose_net_rgbd import CrossModalAttention
    from oracle import resnet as OR
    warnings.simplefilter("ignore")
    torch.manual_seed(0)
    mod = CrossModalAttention(2048, 8, 0.1)
    P = {"cross_attention." + k: v.clone().requires_grad_(True) for k, v in mod.state_dict().items()}
    mod = mod.cuda().eval()
    g = torch.Generator().manual_seed(4)
    r, d = torch.randn(4, 2048, generator=g), torch.randn(4, 2048, generator=g)
    rd, dd = r.cuda().requires_grad_(True), d.cuda().requires_grad_(True)
    out = mod(rd, dd)
    rr, dr = r.clone().requires_grad_(True), d.clone().requires_grad_(True)
    ref = OR.cross_attention(rr, dr, P)
    _close(out, ref, 1e-4, "out")
    w = torch.randn(4, 2048, generator=g)
    (out * w.cuda()).sum().backward()
    (ref * w).sum().backward()
    _close(rd.grad, rr.grad, 1e-4, "d rgb_feat")
    _close(dd.grad, dr.grad, 1e-4, "d depth_feat")
    named = dict(mod.named_parameters())
    for k, v in P.items():
        _close(named[k[len("cross_attention."):]].grad, v.grad, 1e-4, k)
