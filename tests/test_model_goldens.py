"""The reference's four PoseNet classes around the trunk, pinned by a fixture the
reference itself produced (tools/gen_goldens.py gen_models -> tests/golden/models.npz).

The reference models were run end to end with a plain-torch trunk stand-in (not
torchvision, which is absent); the fixture records the (B, 2048) features the
stand-in handed the reference's own code, and everything downstream of them:
the BN1d / LayerNorm heads and fusion MLP, CrossModalAttention, the quaternion
normalisations (F.normalize and q/(||q||+1e-8)), the z-CNN + z-MLP of
PoseNetRGBGeometric (run on the real input image), both pinholes, PoseLoss(1, 10)
and the backward into the features and every reference-owned parameter, in eval
mode and in train mode (Dropout modules in eval, BN batch statistics), plus the
BN running statistics after the step and the reference constructor's own init
constants.  Head parameters come from a seeded generator (tests/synth.py
head_weights); inputs from tests/synth.py model_inputs -- both regenerated here
and checked against the checksums stored in the fixture.

CPU: the oracle (oracle/resnet.py, trunk hook `features=`) against the fixture.
GPU: the drop-in modules (HeadEngine / FusionEngine / the z-CNN TrunkEngine / the
pinhole kernels, fp32) with the recorded features in place of the ResNet50 trunk.
The trunk itself stays parity-unpinned (Oracle)."""
import os

import numpy as np
import pytest
import torch

from oracle import pose_loss as OP
from oracle import resnet as OR
from tests.synth import TRUNK_PREFIXES, head_weights, model_inputs, tensor_checksum

B = 8
INPUT_SEED = 4242
WEIGHT_SEED = {"PoseNetRGB": 101, "PoseNetRGBGeometric": 102, "PoseNetRGBD": 103, "PoseNetRGBDGeometric": 104}
TRUNKS = {"PoseNetRGB": ("backbone",), "PoseNetRGBGeometric": ("rgb_backbone",),
          "PoseNetRGBD": ("rgb_backbone", "depth_backbone"), "PoseNetRGBDGeometric": ("backbone",)}
NAMES = list(TRUNKS)


@pytest.fixture(scope="module")
def fx():
    d = np.load(os.path.join(os.path.dirname(__file__), "golden", "models.npz"))
    return {k: d[k] for k in d.files}


@pytest.fixture(scope="module")
def inputs(fx):
    inp = model_inputs(B, INPUT_SEED)
    for k, v in inp.items():
        # the generator reproduces the fixture's inputs (torch's CPU RNG stream is stable)
        np.testing.assert_array_equal(np.asarray(tensor_checksum(v)), fx[f"inputs/checksum/{k}"], err_msg=k)
    for k in ("bbox", "K", "gt_rot", "gt_trans"):
        np.testing.assert_array_equal(inp[k].numpy(), fx[f"inputs/{k}"])
    return inp


def _model_cls(name):
    import importlib
    mod = {"PoseNetRGB": "pose_net_rgb", "PoseNetRGBGeometric": "pose_net_rgb_geometric",
           "PoseNetRGBD": "pose_net_rgbd", "PoseNetRGBDGeometric": "pose_net_rgbd_geometric"}[name]
    return getattr(importlib.import_module("models." + mod), name)


_SD_CACHE = {}


def _state(name, fx):
    """The drop-in model's state_dict with the fixture's seeded parameters loaded
    (the generator runs over OUR key names and shapes: equal checksums also prove
    the reference-owned layers have the reference's keys and shapes)."""
    if name not in _SD_CACHE:
        torch.manual_seed(0)
        m = _model_cls(name)(pretrained=False)
        sd = {k: v.clone() for k, v in m.state_dict().items()}
        gen = head_weights({k: tuple(v.shape) for k, v in sd.items()}, WEIGHT_SEED[name])
        np.testing.assert_array_equal(np.asarray([tensor_checksum(gen[k]) for k in sorted(gen)]),
                                      fx[f"{name}/weights_checksum"])
        sd.update(gen)
        _SD_CACHE[name] = (sd, gen)
    return _SD_CACHE[name]


def _close(got, ref, rtol, what):
    got = np.asarray(got, np.float64)
    ref = np.asarray(ref, np.float64)
    assert got.shape == ref.shape, (what, got.shape, ref.shape)
    scale = np.abs(ref).max() + 1e-30
    err = np.abs(got - ref)
    assert (err <= rtol * np.abs(ref) + rtol * scale).all(), f"{what}: max err {err.max():.3e} (scale {scale:.3e})"


def _check_grads(fx, name, grads, rtol):
    """grads: {param name: full gradient array}; against first rows, norm and sum."""
    pre = f"{name}/train/grad/"
    keys = [k[len(pre):] for k in fx if k.startswith(pre)]
    assert keys and set(keys) == set(grads), sorted(set(keys) ^ set(grads))
    norms = {k: float(fx[f"{name}/train/gradnorm/{k}"]) for k in keys}
    top = max(norms.values())
    for k in keys:
        g = np.asarray(grads[k], np.float64)
        ref = fx[pre + k]
        if norms[k] < 1e-3 * top:
            # the bias of a layer followed by a batch-statistics BatchNorm: its true
            # gradient is 0 (the BN removes the per-channel mean), so the reference
            # holds rounding noise (norms 1e-8..3e-4 against >= 0.04 for every other
            # gradient); ours must be noise of the same order, not a value
            assert np.linalg.norm(g) < 1e-3 * top, (k, np.linalg.norm(g), norms[k])
            continue
        _close(g[:ref.shape[0]] if g.ndim >= 2 else g, ref, rtol, f"grad {k}")
        nrm = float(fx[f"{name}/train/gradnorm/{k}"])
        np.testing.assert_allclose(np.linalg.norm(g), nrm, rtol=rtol, err_msg=f"grad norm {k}")
        assert abs(g.sum() - float(fx[f"{name}/train/gradsum/{k}"])) <= rtol * (nrm * np.sqrt(g.size) + 1e-30), k


def _oracle_forward(name, P, inp, training, feats):
    if name == "PoseNetRGB":
        return OR.forward_rgb(P, inp["rgb"], training, features=feats)
    if name == "PoseNetRGBGeometric":
        return OR.forward_rgb_geometric(P, inp["rgb"], inp["bbox"], inp["K"], training, features=feats)
    if name == "PoseNetRGBD":
        return OR.forward_rgbd(P, inp["rgb"], inp["depth"], training=training, features=feats)
    return OR.forward_rgbd_geometric(P, inp["rgb"], inp["depth"], inp["depth_raw"], inp["bbox"], inp["K"],
                                     training, features=feats)


@pytest.mark.parametrize("name", NAMES)
def test_oracle_models_vs_reference(fx, inputs, name):
    """The oracle's restatement of every reference-owned layer, fp32: outputs 1e-5,
    gradients 1e-4 (thread-count-dependent summation order through BN backward)."""
    sd, gen = _state(name, fx)
    P = {k: v.clone() for k, v in sd.items()}
    feats = {t: torch.from_numpy(fx[f"{name}/eval/feat/{t}"]) for t in TRUNKS[name]}
    with torch.no_grad():
        rot, trans = _oracle_forward(name, P, inputs, False, feats)
    _close(rot, fx[f"{name}/eval/rot"], 1e-5, "eval rotation")
    _close(trans, fx[f"{name}/eval/trans"], 1e-5, "eval translation")
    if name == "PoseNetRGBGeometric":
        with torch.no_grad():
            _close(OR.z_backbone(inputs["rgb"], P, False), fx[f"{name}/eval/zfeat"], 1e-5, "eval z-CNN")
    # train mode: batch statistics, running-stat updates, PoseLoss(1, 10) backward
    P = {}
    for k, v in sd.items():
        v = v.clone()
        if v.is_floating_point() and "running" not in k and not k.startswith(TRUNK_PREFIXES):
            v.requires_grad_(True)
        P[k] = v
    feats = {t: torch.from_numpy(fx[f"{name}/train/feat/{t}"]).requires_grad_(True) for t in TRUNKS[name]}
    zf = {}
    if name == "PoseNetRGBGeometric":
        orig = OR.z_backbone

        def zhook(x, P_, training):
            y = orig(x, P_, training)
            y.retain_grad()
            zf["z"] = y
            return y
        OR.z_backbone = zhook
    try:
        rot, trans = _oracle_forward(name, P, inputs, True, feats)
    finally:
        if zf or name == "PoseNetRGBGeometric":
            OR.z_backbone = orig
    loss = OP.pose_loss(rot, trans, inputs["gt_rot"], inputs["gt_trans"], 1.0, 10.0)
    loss.backward()
    _close(rot.detach(), fx[f"{name}/train/rot"], 1e-5, "train rotation")
    _close(trans.detach(), fx[f"{name}/train/trans"], 1e-5, "train translation")
    _close(loss.detach(), fx[f"{name}/train/loss"], 1e-5, "loss")
    for t in TRUNKS[name]:
        _close(feats[t].grad, fx[f"{name}/train/feat_grad/{t}"], 1e-5, f"feature grad {t}")
    if zf:
        _close(zf["z"].detach(), fx[f"{name}/train/zfeat"], 1e-5, "train z-CNN")
        _close(zf["z"].grad, fx[f"{name}/train/zfeat_grad"], 1e-5, "z-CNN feature grad")
    _check_grads(fx, name, {k: P[k].grad.numpy() for k in gen if P[k].requires_grad}, 1e-4)
    pre = f"{name}/train/state/"
    for k in [k[len(pre):] for k in fx if k.startswith(pre)]:
        if k.endswith("num_batches_tracked"):
            assert int(P[k]) == int(fx[pre + k]), k
        else:
            _close(P[k], fx[pre + k], 1e-5, k)


@pytest.mark.parametrize("name", NAMES)
def test_init_constants_match_reference(fx, name):
    """The reference constructor's own init (pose_net_rgb.py:53-54,
    pose_net_rgb_geometric.py:68, pose_net_rgbd.py:107-116) on the drop-in modules."""
    torch.manual_seed(0)
    m = _model_cls(name)(pretrained=False)
    if f"{name}/init/trans_bias" in fx:
        np.testing.assert_array_equal(m.trans_head[-1].bias.detach().numpy(), fx[f"{name}/init/trans_bias"])
    if f"{name}/init/z_bias" in fx:
        np.testing.assert_array_equal(m.z_predictor[-1].bias.detach().numpy(), fx[f"{name}/init/z_bias"])
    if name == "PoseNetRGBD":
        for seqn in ("fusion", "rot_head", "trans_head"):
            for i, layer in enumerate(getattr(m, seqn)):
                if not isinstance(layer, torch.nn.Linear):
                    continue
                amax, std = fx[f"{name}/init/{seqn}.{i}/absmax_std"]
                w = layer.weight.detach().double()
                bound = (6.0 / (w.shape[0] + w.shape[1])) ** 0.5          # xavier-uniform
                assert w.abs().max().item() <= bound and amax <= bound
                # both sample stds within 5 sigma of the xavier-uniform std bound / sqrt(3)
                tol = 5.0 / (2.0 * w.numel()) ** 0.5 * bound / 3 ** 0.5
                for s_ in (w.std().item(), std):
                    assert abs(s_ - bound / 3 ** 0.5) <= tol, (seqn, i, s_)
                if seqn == "trans_head" and i == 6:
                    continue
                assert float(fx[f"{name}/init/{seqn}.{i}/bias_absmax"]) == 0.0
                assert layer.bias.abs().max().item() == 0.0


# ---------------------------------------------------------------------------- GPU

def _gpu_model(name, fx):
    sd, gen = _state(name, fx)
    torch.manual_seed(0)
    m = _model_cls(name)(pretrained=False)
    m.load_state_dict(sd)
    m = m.cuda()
    return m, gen


def _hook_trunks(m, feats):
    """Replace the ResNet50 trunk runs by the recorded features (the z-CNN still
    runs on its TrunkEngine)."""
    orig = m._run_trunk

    def run(name, seq, x, in_channels, kind="resnet50"):
        if kind == "resnet50":
            return feats[name]
        return orig(name, seq, x, in_channels, kind)
    m._run_trunk = run


def _model_args(name, cin):
    return {"PoseNetRGB": ("rgb",), "PoseNetRGBGeometric": ("rgb", "bbox", "K"), "PoseNetRGBD": ("rgb", "depth"),
            "PoseNetRGBDGeometric": ("rgb", "depth", "depth_raw", "bbox", "K")}[name]


@pytest.mark.gpu
@pytest.mark.parametrize("name", NAMES)
def test_dropin_models_vs_reference(fx, inputs, name):
    """The drop-in modules' HIP heads / fusion / z-CNN / pinholes (fp32) against the
    reference's own model code, 1e-4 relative."""
    from models.pose_loss import PoseLoss
    m, gen = _gpu_model(name, fx)
    cin = {k: v.cuda() for k, v in inputs.items()}
    args = [cin[a] for a in _model_args(name, cin)]
    # eval
    m.eval()
    _hook_trunks(m, {t: torch.from_numpy(fx[f"{name}/eval/feat/{t}"]).cuda() for t in TRUNKS[name]})
    with torch.no_grad():
        rot, trans = m(*args)
    _close(rot.cpu(), fx[f"{name}/eval/rot"], 1e-4, "eval rotation")
    _close(trans.cpu(), fx[f"{name}/eval/trans"], 1e-4, "eval translation")
    # train, Dropout modules in eval
    m.train()
    for mod in m.modules():
        if isinstance(mod, torch.nn.Dropout):
            mod.eval()
    feats = {t: torch.from_numpy(fx[f"{name}/train/feat/{t}"]).cuda().requires_grad_(True) for t in TRUNKS[name]}
    _hook_trunks(m, feats)
    rot, trans = m(*args)
    loss = PoseLoss(1.0, 10.0, "geodesic")(rot, trans, cin["gt_rot"], cin["gt_trans"])
    loss.backward()
    _close(rot.detach().cpu(), fx[f"{name}/train/rot"], 1e-4, "train rotation")
    _close(trans.detach().cpu(), fx[f"{name}/train/trans"], 1e-4, "train translation")
    _close(loss.detach().cpu(), fx[f"{name}/train/loss"], 1e-4, "loss")
    for t in TRUNKS[name]:
        _close(feats[t].grad.cpu(), fx[f"{name}/train/feat_grad/{t}"], 1e-4, f"feature grad {t}")
    named = dict(m.named_parameters())
    _check_grads(fx, name, {k: named[k].grad.cpu().numpy() for k in gen if k in named}, 1e-4)
    sd = m.state_dict()
    pre = f"{name}/train/state/"
    for k in [k[len(pre):] for k in fx if k.startswith(pre)]:
        if k.endswith("num_batches_tracked"):
            assert int(sd[k]) == int(fx[pre + k]), k
        else:
            _close(sd[k].cpu(), fx[pre + k], 1e-4, k)
