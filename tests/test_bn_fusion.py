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
