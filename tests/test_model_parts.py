"""The reference's own torchvision-free model code, pinned by fixtures the
reference itself produced (tools/gen_goldens.py -> tests/golden/model_parts.npz):
CrossModalAttention (pose_net_rgbd.py:8-35, eval mode) with its input and
parameter gradients, PoseNetRGBDGeometric._compute_pinhole_translation
(pose_net_rgbd_geometric.py:56-85) and PoseNetRGBGeometric._compute_pinhole_translation
(pose_net_rgb_geometric.py:93-109) with its z gradient.
CPU: the oracle's restatements against the fixtures.  GPU: the drop-in modules /
HIP kernels against the same fixtures (fp32, 1e-4 relative; pinhole: the exact
fp32 formula, 1e-6)."""
import numpy as np
import pytest
import torch

from oracle import resnet as OR
from tests.synth import xattn_weights

CASES = {"xattn": 2048 + 8, "xattn_small": 64 + 4}


@pytest.fixture(scope="module")
def parts():
    import os
    d = np.load(os.path.join(os.path.dirname(__file__), "golden", "model_parts.npz"))
    return {k: d[k] for k in d.files}


def _weights(parts, name):
    D = parts[f"{name}/rgb_feat"].shape[1]
    sd = xattn_weights(D, CASES[name])
    chk = np.asarray([float(v.numpy().astype(np.float64).sum()) for v in sd.values()])
    # the generator reproduces the fixture's weights (torch's CPU RNG stream is stable)
    np.testing.assert_array_equal(chk, parts[f"{name}/weights_checksum"])
    return sd


def _close(got, ref, rtol, what):
    got = np.asarray(got, np.float64)
    ref = np.asarray(ref, np.float64)
    scale = np.abs(ref).max() + 1e-30
    err = np.abs(got - ref)
    assert (err <= rtol * np.abs(ref) + rtol * scale).all(), f"{what}: max err {err.max():.3e} (scale {scale:.3e})"


@pytest.mark.parametrize("name", list(CASES))
def test_oracle_cross_attention_vs_reference(parts, name):
    sd = _weights(parts, name)
    P = {f"cross_attention.{k}": v.clone().requires_grad_(True) for k, v in sd.items()}
    r = torch.from_numpy(parts[f"{name}/rgb_feat"]).requires_grad_(True)
    d = torch.from_numpy(parts[f"{name}/depth_feat"]).requires_grad_(True)
    y = OR.cross_attention(r, d, P, heads=int(parts[f"{name}/heads"]))
    (y * torch.from_numpy(parts[f"{name}/dout"])).sum().backward()
    _close(y.detach(), parts[f"{name}/out"], 1e-5, "out")
    _close(r.grad, parts[f"{name}/grad_rgb"], 1e-5, "grad rgb")
    _close(d.grad, parts[f"{name}/grad_depth"], 1e-5, "grad depth")
    for k, v in P.items():
        k = k[len("cross_attention."):]
        g = v.grad.numpy()
        _close(g[:16] if g.ndim == 2 else g, parts[f"{name}/grad/{k}"], 1e-5, f"grad {k}")
        np.testing.assert_allclose(np.linalg.norm(g.astype(np.float64)), parts[f"{name}/gradnorm/{k}"], rtol=1e-5)


def test_oracle_pinholes_vs_reference(parts):
    dr, bb, K = (torch.from_numpy(parts[f"pin_depth/{k}"]) for k in ("depth_raw", "bbox", "K"))
    np.testing.assert_array_equal(OR.pinhole_rgbd_geometric(dr, bb, K).numpy(), parts["pin_depth/out_Kb"])
    np.testing.assert_array_equal(OR.pinhole_rgbd_geometric(dr, bb, K[5]).numpy(), parts["pin_depth/out_K2"])
    z = torch.from_numpy(parts["pin_z/z"]).requires_grad_(True)
    bz, Kz = torch.from_numpy(parts["pin_z/bbox"]), torch.from_numpy(parts["pin_z/K"])
    t = OR.pinhole_rgb_geometric(z, bz, Kz)
    (t * torch.from_numpy(parts["pin_z/dout"])).sum().backward()
    np.testing.assert_array_equal(t.detach().numpy(), parts["pin_z/out_Kb"])
    np.testing.assert_array_equal(z.grad.numpy(), parts["pin_z/grad_z"])
    np.testing.assert_array_equal(OR.pinhole_rgb_geometric(z.detach(), bz, Kz[7]).numpy(), parts["pin_z/out_K2"])


@pytest.mark.gpu
@pytest.mark.parametrize("name", list(CASES))
def test_cross_attention_module_vs_reference(parts, name):
    from models.pose_net_rgbd import CrossModalAttention
    sd = _weights(parts, name)
    D = parts[f"{name}/rgb_feat"].shape[1]
    att = CrossModalAttention(D, num_heads=int(parts[f"{name}/heads"]), dropout=0.1)
    att.load_state_dict(sd)
    att = att.cuda().eval()
    r = torch.from_numpy(parts[f"{name}/rgb_feat"]).cuda().requires_grad_(True)
    d = torch.from_numpy(parts[f"{name}/depth_feat"]).cuda().requires_grad_(True)
    y = att(r, d)
    (y * torch.from_numpy(parts[f"{name}/dout"]).cuda()).sum().backward()
    _close(y.detach().cpu(), parts[f"{name}/out"], 1e-4, "out")
    _close(r.grad.cpu(), parts[f"{name}/grad_rgb"], 1e-4, "grad rgb")
    _close(d.grad.cpu(), parts[f"{name}/grad_depth"], 1e-4, "grad depth")
    for k, p in att.named_parameters():
        g = p.grad.cpu().numpy()
        _close(g[:16] if g.ndim == 2 else g, parts[f"{name}/grad/{k}"], 1e-4, f"grad {k}")
        np.testing.assert_allclose(np.linalg.norm(g.astype(np.float64)), parts[f"{name}/gradnorm/{k}"], rtol=1e-4)


@pytest.mark.gpu
def test_pinhole_methods_vs_reference(parts):
    """The drop-in models' own _compute_pinhole_translation (HIP kernels)."""
    from models.pose_net_rgb_geometric import PoseNetRGBGeometric
    from models.pose_net_rgbd_geometric import PoseNetRGBDGeometric
    dr, bb, K = (torch.from_numpy(parts[f"pin_depth/{k}"]).cuda() for k in ("depth_raw", "bbox", "K"))
    pin = PoseNetRGBDGeometric._compute_pinhole_translation
    _close(pin(None, dr, bb, K).cpu(), parts["pin_depth/out_Kb"], 1e-6, "pinhole depth, K per sample")
    _close(pin(None, dr, bb, K[5]).cpu(), parts["pin_depth/out_K2"], 1e-6, "pinhole depth, one K")
    pinz = PoseNetRGBGeometric._compute_pinhole_translation
    z = torch.from_numpy(parts["pin_z/z"]).cuda().requires_grad_(True)
    bz, Kz = torch.from_numpy(parts["pin_z/bbox"]).cuda(), torch.from_numpy(parts["pin_z/K"]).cuda()
    t = pinz(None, z, bz, Kz)
    (t * torch.from_numpy(parts["pin_z/dout"]).cuda()).sum().backward()
    _close(t.detach().cpu(), parts["pin_z/out_Kb"], 1e-6, "pinhole z")
    _close(z.grad.cpu(), parts["pin_z/grad_z"], 1e-6, "pinhole z grad")
    _close(pinz(None, z.detach(), bz, Kz[7]).cpu(), parts["pin_z/out_K2"], 1e-6, "pinhole z, one K")
