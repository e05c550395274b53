"""Head kernels (fp32 nn.Linear / BatchNorm1d of the pose heads) against a plain
PyTorch fp32 reference of the same op: the MFMA skinny GEMM behind
pose6d_gemm_f32 (forward x W^T and data gradient dy W), the fused weight + bias
gradient pose6d_linear_wgrad, and BatchNorm1d(+ReLU) forward/backward."""
import pytest
import torch

pytestmark = pytest.mark.gpu

SHAPES = [(32, 2048, 1024), (32, 1024, 512), (32, 512, 4), (4, 64, 16), (1, 20, 7), (32, 4, 512), (17, 4096, 1024)]


def _dev():
    return torch.device("cuda")


@pytest.mark.parametrize("M,K,N", SHAPES)
def test_linear_forward_and_dgrad(M, K, N):
    from pose6d._lib import call, stream
    g = torch.Generator(device="cuda").manual_seed(M * 7 + N)
    x = torch.randn(M, K, device=_dev(), generator=g)
    w = torch.randn(N, K, device=_dev(), generator=g) * 0.05
    b = torch.randn(N, device=_dev(), generator=g)
    y = torch.empty(M, N, device=_dev())
    call("gemm_f32", x, K, 1, w, 1, K, y, N, b, M, N, K, 1.0, 0.0, None, 0, stream())
    ref = x.double() @ w.double().T + b.double()
    torch.testing.assert_close(y.double(), ref, rtol=1e-5, atol=1e-5 * ref.abs().max().item())
    # data gradient dx = dy W, accumulated onto an existing dx (beta = 1)
    dy = torch.randn(M, N, device=_dev(), generator=g)
    dx = torch.randn(M, K, device=_dev(), generator=g)
    ref = dy.double() @ w.double() + dx.double()
    call("gemm_f32", dy, N, 1, w, K, 1, dx, K, None, M, K, N, 1.0, 1.0, None, 0, stream())
    torch.testing.assert_close(dx.double(), ref, rtol=1e-5, atol=1e-5 * ref.abs().max().item())


def test_linear_strided_rows():
    """Row strides (the RGBD concatenation is written in place): x rows of 4096
    floats, the second half used as a (B, 2048) operand."""
    from pose6d._lib import call, stream
    g = torch.Generator(device="cuda").manual_seed(3)
    big = torch.randn(32, 4098, device=_dev(), generator=g)
    x = big[:, 2:2050]                       # 8-byte aligned only: scalar-load path
    w = torch.randn(256, 2048, device=_dev(), generator=g) * 0.05
    y = torch.empty(32, 256, device=_dev())
    call("gemm_f32", x, 4098, 1, w, 1, 2048, y, 256, None, 32, 256, 2048, 1.0, 0.0, None, 0, stream())
    ref = x.double() @ w.double().T
    torch.testing.assert_close(y.double(), ref, rtol=1e-5, atol=1e-5 * ref.abs().max().item())


@pytest.mark.parametrize("Bn,K,N", [(32, 2048, 1024), (32, 512, 4), (5, 7, 3), (32, 4096, 1024)])
@pytest.mark.parametrize("acc", [0, 1])
def test_linear_wgrad(Bn, K, N, acc):
    from pose6d._lib import call, stream
    g = torch.Generator(device="cuda").manual_seed(Bn + K + N)
    dy = torch.randn(Bn, N, device=_dev(), generator=g)
    x = torch.randn(Bn, K, device=_dev(), generator=g)
    dw = torch.randn(N, K, device=_dev(), generator=g)
    db = torch.randn(N, device=_dev(), generator=g)
    ref_w = dy.double().T @ x.double() + (dw.double() if acc else 0)
    ref_b = dy.double().sum(0) + (db.double() if acc else 0)
    call("linear_wgrad", dy, N, x, K, dw, db, N, K, Bn, acc, stream())
    torch.testing.assert_close(dw.double(), ref_w, rtol=1e-5, atol=1e-5 * ref_w.abs().max().item())
    torch.testing.assert_close(db.double(), ref_b, rtol=1e-5, atol=1e-5 * ref_b.abs().max().item())


@pytest.mark.parametrize("M,C", [(32, 1024), (32, 512), (2, 70), (33, 65)])
def test_bn1d_relu_fwd_bwd(M, C):
    from pose6d._lib import call, stream
    g = torch.Generator(device="cuda").manual_seed(M + C)
    x = torch.randn(M, C, device=_dev(), generator=g) * 2 + 0.5
    gamma = torch.rand(C, device=_dev(), generator=g) + 0.5
    beta = torch.randn(C, device=_dev(), generator=g)
    rm, rv = torch.zeros(C, device=_dev()), torch.ones(C, device=_dev())
    nbt = torch.zeros(1, device=_dev(), dtype=torch.int64)
    y = torch.empty_like(x)
    sm, si = torch.empty(C, device=_dev()), torch.empty(C, device=_dev())
    call("bn1d_fwd", x, y, M, C, gamma, beta, rm, rv, nbt, 0.1, 1e-5, 1, 1, 0.0, None, 0, None, sm, si, stream())
    xr = x.double().requires_grad_(True)
    ref = torch.relu(torch.nn.functional.batch_norm(xr, None, None, gamma.double(), beta.double(), True, 0.1, 1e-5))
    torch.testing.assert_close(y.double(), ref, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(rm.double(), 0.1 * x.double().mean(0), rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(rv.double(), 0.9 + 0.1 * x.double().var(0, unbiased=True), rtol=1e-5, atol=1e-6)
    assert int(nbt.item()) == 1
    dy = torch.randn(M, C, device=_dev(), generator=g)
    ref.backward(dy.double())
    dx = torch.empty_like(x)
    dg, db = torch.empty(C, device=_dev()), torch.empty(C, device=_dev())
    call("bn1d_bwd", dy, x, y, M, C, gamma, sm, si, 1, 1, 0.0, None, dx, dg, db, 0, stream())
    # dx = gamma * invstd * (dy - mean(dy) - xhat * mean(dy * xhat)): cancels to ~0 for tiny
    # batches, so the absolute tolerance is scaled by gamma * invstd * |dy|, not by |dx|
    scale = ((gamma * si).max() * dy.abs().max()).item()
    torch.testing.assert_close(dx.double(), xr.grad, rtol=1e-4, atol=1e-5 * scale)


def test_geo_head_loss_matches_separate_calls():
    """pose6d_geo_head_loss == rownorm_fwd + pinhole_depth + pose_loss_fwd/_bwd + rownorm_bwd (same formulas;
    the compiler may contract the normalize-backward differently: 1e-6)."""
    from pose6d._lib import call, stream
    from bench import synth_batch
    B = 32
    _, depth_raw, bbox, K, gr, gt = synth_batch(B, "cuda", seed=9)
    raw = torch.randn(B, 4, device="cuda") * 3
    raw[3] = 0.0                               # zero-norm row (F.normalize eps branch)
    f = lambda *s: torch.empty(*s, device="cuda")
    rot, trans, loss, draw, dtr = f(B, 4), f(B, 3), f(()), f(B, 4), f(B, 3)
    call("geo_head_loss", raw, depth_raw, 224, 224, bbox, K, 1, gr, gt, B, 1.0, 10.0, 0, rot, trans, loss, draw, dtr,
         stream())
    rot2, trans2, loss2, drot2, draw2, dtr2 = f(B, 4), f(B, 3), f(()), f(B, 4), f(B, 4), f(B, 3)
    one = torch.ones((), device="cuda")
    call("rownorm_fwd", raw, rot2, B, 4, 0, stream())
    call("pinhole_depth", depth_raw, 224, 224, bbox, K, 1, B, trans2, stream())
    call("pose_loss_fwd", rot2, trans2, gr, gt, B, 1.0, 10.0, 0, loss2, stream())
    call("pose_loss_bwd", rot2, trans2, gr, gt, B, 1.0, 10.0, 0, one, drot2, dtr2, stream())
    call("rownorm_bwd", raw, drot2, draw2, B, 4, 0, stream())
    torch.cuda.synchronize()
    for a, b in ((rot, rot2), (trans, trans2), (loss, loss2), (dtr, dtr2)):
        assert torch.equal(a, b)
    torch.testing.assert_close(draw, draw2, rtol=1e-6, atol=1e-9)


def test_eval_head_backward_through_autograd():
    """Eval-mode head (running-stat BatchNorm1d, no dropout) differentiated through
    autograd -- e.g. heads fine-tuned under model.eval(): the Linear + BatchNorm1d
    eval fusion must not run there (grad mode is off inside autograd.Function.forward,
    yet a backward follows).  Output, input and parameter gradients vs torch fp32."""
    from pose6d import autograd
    from pose6d.head import HeadEngine
    torch.manual_seed(0)
    seq = torch.nn.Sequential(torch.nn.Linear(256, 128), torch.nn.BatchNorm1d(128), torch.nn.ReLU(),
                              torch.nn.Dropout(0.3), torch.nn.Linear(128, 4)).cuda().eval()
    g = torch.Generator().manual_seed(21)
    bn = seq[1]
    bn.running_mean.copy_(torch.randn(128, generator=g).cuda() * 0.1)
    bn.running_var.copy_(torch.rand(128, generator=g).cuda() + 0.5)
    bn.weight.data.copy_(torch.rand(128, generator=g).cuda() + 0.5)
    x = torch.randn(32, 256, generator=g).cuda().requires_grad_(True)
    dy = torch.randn(32, 4, generator=g).cuda()
    eng = HeadEngine(seq)
    out = autograd.run(eng, x, False, list(seq.parameters()))
    grads = torch.autograd.grad(out, [x] + list(seq.parameters()), dy)
    xr = x.detach().clone().requires_grad_(True)
    ref = seq(xr)
    rgrads = torch.autograd.grad(ref, [xr] + list(seq.parameters()), dy)
    torch.testing.assert_close(out, ref, rtol=1e-5, atol=1e-5)
    for a, b in zip(grads, rgrads):
        torch.testing.assert_close(a, b, rtol=1e-4, atol=1e-5 * b.abs().max().item())
