"""Drop-in PoseNet models: structure (CPU) and forward/backward parity against the
oracle's torch-CPU fp32 restatement (GPU)."""
import warnings

import numpy as np
import pytest
import torch

from oracle import pose_loss as OP
from oracle import resnet as OR

# SURVEY.md §8a (measured on the reference with torchvision's ResNet50)
EXPECTED = {
    "PoseNetRGB": (37162567, 354),
    "PoseNetRGBGeometric": (26603333, 368),
    "PoseNetRGBDGeometric": (26136132, 334),
}


def _models():
    from models.pose_net_rgb import PoseNetRGB
    from models.pose_net_rgb_geometric import PoseNetRGBGeometric
    from models.pose_net_rgbd_geometric import PoseNetRGBDGeometric
    return {"PoseNetRGB": PoseNetRGB, "PoseNetRGBGeometric": PoseNetRGBGeometric,
            "PoseNetRGBDGeometric": PoseNetRGBDGeometric}


@pytest.mark.parametrize("name", list(EXPECTED))
def test_structure_matches_reference(name):
    torch.manual_seed(0)
    m = _models()[name](pretrained=False)
    n, keys = EXPECTED[name]
    assert sum(p.numel() for p in m.parameters()) == n
    sd = m.state_dict()
    assert len(sd) == keys
    assert not any(k.startswith("_p6") for k in sd)
    # torchvision naming inside the Sequential trunk
    pre = "backbone" if "backbone.0.weight" in sd else "rgb_backbone"
    for k in (f"{pre}.0.weight", f"{pre}.1.running_var", f"{pre}.4.0.downsample.0.weight",
              f"{pre}.7.2.conv3.weight", f"{pre}.7.2.bn3.num_batches_tracked"):
        assert k in sd, k
    assert sd[f"{pre}.0.weight"].shape == (64, 3, 7, 7)


def _oracle_forward(name, P, inputs, training):
    if name == "PoseNetRGB":
        return OR.forward_rgb(P, inputs["rgb"], training)
    if name == "PoseNetRGBGeometric":
        return OR.forward_rgb_geometric(P, inputs["rgb"], inputs["bbox"], inputs["K"], training)
    return OR.forward_rgbd_geometric(P, inputs["rgb"], inputs["depth"], inputs["depth_raw"], inputs["bbox"],
                                     inputs["K"], training)


def _model_forward(name, m, inp):
    if name == "PoseNetRGB":
        return m(inp["rgb"])
    if name == "PoseNetRGBGeometric":
        return m(inp["rgb"], inp["bbox"], inp["K"])
    return m(inp["rgb"], inp["depth"], inp["depth_raw"], inp["bbox"], inp["K"])


def _inputs(B, H, g):
    K = torch.zeros(B, 3, 3)
    K[:, 0, 0] = K[:, 1, 1] = 800.0
    K[:, 0, 2] = K[:, 1, 2] = 112.0
    K[:, 2, 2] = 1
    return {"rgb": torch.randn(B, 3, H, H, generator=g), "depth": torch.rand(B, 1, H, H, generator=g),
            "depth_raw": torch.rand(B, max(H, 224), max(H, 224), generator=g) + 0.3,
            "bbox": torch.rand(B, 2, generator=g) * 200, "K": K,
            "gt_rot": torch.nn.functional.normalize(torch.randn(B, 4, generator=g), dim=1),
            "gt_trans": torch.randn(B, 3, generator=g) * 0.1 + torch.tensor([0, 0, .8])}


@pytest.mark.parametrize("name", list(EXPECTED))
def test_oracle_runs_on_model_state_dict(name):
    """The oracle consumes the drop-in model's state_dict names (CPU, tiny input)."""
    torch.manual_seed(0)
    m = _models()[name](pretrained=False)
    P = {k: v.clone() for k, v in m.state_dict().items()}
    g = torch.Generator().manual_seed(1)
    rot, trans = _oracle_forward(name, P, _inputs(2, 64, g), True)
    assert rot.shape == (2, 4) and trans.shape == (2, 3)


def _close(got, ref, rtol, what):
    got, ref = got.detach().float().cpu(), ref.detach().float().cpu()
    scale = ref.abs().max().item() + 1e-30
    err = (got - ref).abs()
    bad = err > rtol * ref.abs() + rtol * scale
    assert not bool(bad.any()), f"{what}: max err {err.max().item():.3e} vs scale {scale:.3e}"


@pytest.mark.gpu
@pytest.mark.parametrize("name", list(EXPECTED))
def test_train_step_parity_fp32(name):
    """Training-mode forward + PoseLoss(1, 10) + backward in fp32 vs the oracle:
    outputs and loss within 1e-4 relative, parameter gradients within 1e-3 of
    their tensor's scale, BN running statistics updated identically.
    Dropout modules in eval (their RNG differs by construction)."""
    warnings.simplefilter("ignore")
    torch.manual_seed(0)
    m = _models()[name](pretrained=False)
    P = {k: v.clone() for k, v in m.state_dict().items()}
    for k, v in P.items():
        if v.is_floating_point() and "running" not in k:
            v.requires_grad_(True)
    m = m.cuda().train()
    for mod in m.modules():
        if isinstance(mod, torch.nn.Dropout):
            mod.eval()
    g = torch.Generator().manual_seed(1)
    inp = _inputs(4, 224, g)
    cuda_inp = {k: v.cuda() for k, v in inp.items()}
    rot, trans = _model_forward(name, m, cuda_inp)
    loss = OP.pose_loss  # reference formula, applied on device by the drop-in PoseLoss below
    from models.pose_loss import PoseLoss
    crit = PoseLoss(1.0, 10.0, "geodesic")
    L = crit(rot, trans, cuda_inp["gt_rot"], cuda_inp["gt_trans"])
    L.backward()
    rr, tr = _oracle_forward(name, P, inp, True)
    Lr = loss(rr, tr, inp["gt_rot"], inp["gt_trans"], 1.0, 10.0)
    Lr.backward()
    _close(rot, rr, 1e-4, "rotation")
    _close(trans, tr, 1e-4, "translation")
    _close(L, Lr, 1e-4, "loss")
    sd = m.state_dict()
    for k, v in P.items():
        if "running" in k:
            _close(sd[k], v, 1e-4, k)
        elif "num_batches" in k:
            assert int(sd[k]) == int(v), k
    named = dict(m.named_parameters())
    for k, v in P.items():
        if v.grad is None:
            continue
        _close(named[k].grad, v.grad, 1e-3, "grad " + k)
