#!/usr/bin/env python3
"""Generate the golden fixtures under tests/golden/ by running the REAL reference.

Runs only in the build container (where /root/reference exists).  It imports the
reference's own `models/pose_loss.py` and `models/add_loss.py` (both import as-is:
they need only torch/numpy/yaml) and records their outputs on seeded synthetic
inputs.  Nothing from the reference is copied: the fixtures are inputs + outputs.

    python tools/gen_goldens.py            # rewrites tests/golden/*.npz

The reference's `models/pose_net_*.py` import torchvision at module level, which is
absent from this image.  Their torchvision-free parts -- `CrossModalAttention`
(pose_net_rgbd.py:8-35) and both `_compute_pinhole_translation` methods
(pose_net_rgbd_geometric.py:56-85, pose_net_rgb_geometric.py:93-109) -- are run
by importing those files against a `torchvision` placeholder whose every
attribute access RAISES: the module-level import succeeds, and no third-party
arithmetic can enter a fixture (nothing there constructs a model, so nothing asks
for `models.resnet50`).

The four model classes themselves (gen_models -> tests/golden/models.npz) run with
a `torchvision.models` stand-in whose resnet50() is a small plain-torch network with
ResNet's child layout (_StandInResNet): the fixture records the features that
stand-in hands the reference's own code and everything downstream of them, so the
heads, fusion, z-CNN, normalisations and pinholes are pinned while no value depends
on a restatement of torchvision.  The ResNet50 trunk itself stays parity-unpinned
(DESIGN.md "Oracle").

    python tools/gen_goldens.py models     # only tests/golden/models.npz
"""
import importlib.util
import json
import os
import sys
import tempfile
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, REPO)
from tests.synth import write_mesh_dir, LINEMOD_OBJ_IDS, make_poses, grid_mesh, xattn_weights  # noqa: E402

REF = os.environ.get("POSE6D_REFERENCE", "/root/reference")
OUT = os.path.join(REPO, "tests", "golden")


def _load(modname, relpath):
    spec = importlib.util.spec_from_file_location(modname, os.path.join(REF, relpath))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def gen_pose_loss(ref_pl):
    g = torch.Generator().manual_seed(7)
    cases = {}
    B = 32
    gt = torch.nn.functional.normalize(torch.randn(B, 4, generator=g), dim=1)
    cases["random"] = (torch.randn(B, 4, generator=g), torch.randn(B, 3, generator=g) * 0.1 + torch.tensor([0, 0, .8]),
                       gt, torch.randn(B, 3, generator=g) * 0.1 + torch.tensor([0, 0, .8]))
    gt8 = torch.nn.functional.normalize(torch.randn(8, 4, generator=g), dim=1)
    t8 = torch.randn(8, 3, generator=g)
    cases["identical"] = (gt8.clone(), t8.clone(), gt8.clone(), t8.clone())
    cases["antipodal"] = (-gt8.clone() * 3.0, t8 + 0.01, gt8.clone(), t8.clone())
    zr = torch.randn(8, 4, generator=g)
    zr[2] = 0.0
    zr[5] = 1e-20
    cases["zero_norm"] = (zr, t8 * 2, gt8.clone(), t8.clone())
    # orthogonal quaternions: dot == 0 exactly (q2 = [-y, x, -w, z])
    q = gt8.clone()
    orth = torch.stack([-q[:, 1], q[:, 0], -q[:, 3], q[:, 2]], dim=1)
    cases["orthogonal"] = (orth, t8, q, t8 + 0.5)
    cases["single"] = (torch.randn(1, 4, generator=g), torch.randn(1, 3, generator=g), gt8[:1].clone(), t8[:1].clone())
    cases["scaled"] = (gt8 * 1e3 + 1e-3 * torch.randn(8, 4, generator=g), t8, gt8, t8 - 0.25)

    out = {}
    modes = [("geodesic", 1.0, 10.0), ("geodesic", 1.0, 1.0), ("l1", 1.0, 10.0), ("l1", 0.5, 2.0)]
    for name, (pr, pt, gr, gtt) in cases.items():
        out[f"{name}/pred_rot"] = pr.numpy()
        out[f"{name}/pred_trans"] = pt.numpy()
        out[f"{name}/gt_rot"] = gr.numpy()
        out[f"{name}/gt_trans"] = gtt.numpy()
        for mode, wr, wt in modes:
            crit = ref_pl.PoseLoss(rot_weight=wr, trans_weight=wt, rotation_loss=mode)
            a = pr.clone().requires_grad_(True)
            b = pt.clone().requires_grad_(True)
            loss = crit(a, b, gr, gtt)
            loss.backward()
            key = f"{name}/{mode}_{wr:g}_{wt:g}"
            out[key + "/loss"] = np.asarray(loss.detach().numpy(), dtype=np.float32)
            out[key + "/grad_rot"] = a.grad.numpy()
            out[key + "/grad_trans"] = b.grad.numpy()
    np.savez_compressed(os.path.join(OUT, "pose_loss.npz"), **out)
    meta = {"cases": list(cases), "modes": [f"{m}_{a:g}_{b:g}" for m, a, b in modes]}
    with open(os.path.join(OUT, "pose_loss.json"), "w") as f:
        json.dump(meta, f, indent=1)


def _per_point(crit, pred_r, pred_t, gt_r, gt_t, obj_ids):
    """Per-sample ADD / ADD-S, per-point min distance and argmin, following the
    op sequence of add_loss.py:161-189 on the reference's own matrices."""
    pR = crit._quat_to_mat(pred_r)
    gR = crit._quat_to_mat(gt_r)
    add, adds, mins, idxs, valid = [], [], [], [], []
    for i in range(pred_r.shape[0]):
        oid = int(obj_ids[i].item())
        if oid not in crit.points:
            valid.append(0)
            continue
        valid.append(1)
        P = crit.points[oid]
        G = torch.mm(P, gR[i].T) + gt_t[i]
        Q = torch.mm(P, pR[i].T) + pred_t[i]
        add.append(torch.norm(Q - G, dim=1, p=2).mean().item())
        d = torch.norm(Q.unsqueeze(1) - G.unsqueeze(0), dim=2)
        v, j = d.min(dim=1)
        adds.append(v.mean().item())
        mins.append(v.numpy())
        idxs.append(j.numpy().astype(np.int32))
    return (np.asarray(add, np.float64), np.asarray(adds, np.float64), mins, idxs,
            np.asarray(valid, np.int32), pR.numpy(), gR.numpy())


def gen_add(ref_al):
    out = {}
    with tempfile.TemporaryDirectory() as d:
        write_mesh_dir(d, n_vertices=700, seed=11)
        np.random.seed(1234)
        crit = ref_al.ADDLoss(d, "cpu")
        # loader results (seeded global np.random, add_loss.py:68,78)
        for oid in sorted(crit.points):
            out[f"load/points/{oid}"] = crit.points[oid].numpy()
        out["load/diam_ids"] = np.asarray(sorted(crit.diameters), np.int32)
        out["load/diam_vals"] = np.asarray([crit.diameters[k] for k in sorted(crit.diameters)], np.float64)

        # --- N = 500 (reference default), B = 64 incl. unknown ids ------------
        rng = np.random.default_rng(5)
        ids = np.array([LINEMOD_OBJ_IDS[i % 13] for i in range(60)] + [2, 6, 20, 9], np.int64)
        pr, pt, gr, gt = make_poses(rng, len(ids))
        args = [torch.from_numpy(x) for x in (pr, pt, gr, gt)] + [torch.from_numpy(ids)]
        m = crit.eval_metrics(*args)
        out["n500/pred_rot"], out["n500/pred_trans"], out["n500/gt_rot"], out["n500/gt_trans"] = pr, pt, gr, gt
        out["n500/obj_ids"] = ids
        out["n500/metrics"] = np.asarray([m["add_mean"], m["add_s_mean"], m["add_01d_acc"]], np.float64)
        out["n500/forward"] = np.asarray(crit(*args).item(), np.float64)
        add, adds, mins, idxs, valid, pR, gR = _per_point(crit, *args)
        out["n500/add"], out["n500/adds"], out["n500/valid"] = add, adds, valid
        out["n500/pred_R"], out["n500/gt_R"] = pR, gR
        out["n500/min_dist"] = np.concatenate(mins)
        out["n500/npts"] = np.asarray([len(x) for x in mins], np.int32)
        out["n500/argmin"] = np.concatenate(idxs)

        # --- N = 2000 (BASELINE config 4 size): override the points dict -----
        rng = np.random.default_rng(6)
        for oid in LINEMOD_OBJ_IDS:
            crit.points[oid] = torch.from_numpy((rng.standard_normal((2000, 3)) * 0.04).astype(np.float32))
        ids = np.array([LINEMOD_OBJ_IDS[i % 13] for i in range(26)], np.int64)
        pr, pt, gr, gt = make_poses(rng, len(ids))
        args = [torch.from_numpy(x) for x in (pr, pt, gr, gt)] + [torch.from_numpy(ids)]
        m = crit.eval_metrics(*args)
        for oid in LINEMOD_OBJ_IDS:
            out[f"n2000/points/{oid}"] = crit.points[oid].numpy()
        out["n2000/pred_rot"], out["n2000/pred_trans"], out["n2000/gt_rot"], out["n2000/gt_trans"] = pr, pt, gr, gt
        out["n2000/obj_ids"] = ids
        out["n2000/metrics"] = np.asarray([m["add_mean"], m["add_s_mean"], m["add_01d_acc"]], np.float64)
        out["n2000/forward"] = np.asarray(crit(*args).item(), np.float64)
        add, adds, mins, idxs, valid, _, _ = _per_point(crit, *args)
        out["n2000/add"], out["n2000/adds"], out["n2000/valid"] = add, adds, valid
        out["n2000/min_dist"] = np.concatenate(mins)
        out["n2000/npts"] = np.asarray([len(x) for x in mins], np.int32)
        out["n2000/argmin"] = np.concatenate(idxs)

        # --- ties: integer-mm grid meshes with duplicated vertices ---------------
        rng = np.random.default_rng(8)
        for oid in LINEMOD_OBJ_IDS:
            crit.points[oid] = torch.from_numpy(grid_mesh(rng, 600))
        ids = np.array(LINEMOD_OBJ_IDS, np.int64)
        pr, pt, gr, gt = make_poses(rng, len(ids))
        # exact identity pose for a few samples: every point has distance-0 ties
        pr[:3], pt[:3] = gr[:3], gt[:3]
        pr[3] = -gr[3]  # antipodal quaternion: the same rotation
        pt[3] = gt[3]
        args = [torch.from_numpy(x) for x in (pr, pt, gr, gt)] + [torch.from_numpy(ids)]
        m = crit.eval_metrics(*args)
        for oid in LINEMOD_OBJ_IDS:
            out[f"ties/points/{oid}"] = crit.points[oid].numpy()
        out["ties/pred_rot"], out["ties/pred_trans"], out["ties/gt_rot"], out["ties/gt_trans"] = pr, pt, gr, gt
        out["ties/obj_ids"] = ids
        out["ties/metrics"] = np.asarray([m["add_mean"], m["add_s_mean"], m["add_01d_acc"]], np.float64)
        add, adds, mins, idxs, valid, _, _ = _per_point(crit, *args)
        out["ties/add"], out["ties/adds"], out["ties/valid"] = add, adds, valid
        out["ties/min_dist"] = np.concatenate(mins)
        out["ties/npts"] = np.asarray([len(x) for x in mins], np.int32)
        out["ties/argmin"] = np.concatenate(idxs)

        # --- empty batch / all-unknown ids ---------------------------------------
        args = [torch.zeros(0, 4), torch.zeros(0, 3), torch.zeros(0, 4), torch.zeros(0, 3), torch.zeros(0, dtype=torch.long)]
        m = crit.eval_metrics(*args)
        out["empty/metrics"] = np.asarray([m["add_mean"], m["add_s_mean"], m["add_01d_acc"]], np.float64)
        args = [torch.ones(2, 4), torch.ones(2, 3), torch.ones(2, 4), torch.ones(2, 3), torch.tensor([2, 99])]
        m = crit.eval_metrics(*args)
        out["unknown/metrics"] = np.asarray([m["add_mean"], m["add_s_mean"], m["add_01d_acc"]], np.float64)
        out["unknown/forward"] = np.asarray(crit(*args).item(), np.float64)
    out["symmetric_ids"] = np.asarray(sorted(ref_al.SYMMETRIC_OBJECT_IDS), np.int32)
    np.savez_compressed(os.path.join(OUT, "add_loss.npz"), **out)


class _Refuse(types.ModuleType):
    """torchvision placeholder: importable, unusable."""

    def __getattr__(self, name):
        if name.startswith("__"):
            raise AttributeError(name)
        raise RuntimeError(f"torchvision.{name} is not available: fixtures must not depend on it")


def _load_models():
    """Import the reference's pose_net_* modules with the refusing placeholder."""
    tv = _Refuse("torchvision")
    tvm = _Refuse("torchvision.models")
    saved = {k: sys.modules.get(k) for k in ("torchvision", "torchvision.models")}
    sys.modules["torchvision"], sys.modules["torchvision.models"] = tv, tvm
    object.__setattr__(tv, "models", tvm)
    try:
        rgbd = _load("ref_pose_net_rgbd", "models/pose_net_rgbd.py")
        rgbd_geo = _load("ref_pose_net_rgbd_geometric", "models/pose_net_rgbd_geometric.py")
        rgb_geo = _load("ref_pose_net_rgb_geometric", "models/pose_net_rgb_geometric.py")
    finally:
        for k, v in saved.items():
            if v is None:
                sys.modules.pop(k, None)
            else:
                sys.modules[k] = v
    return rgbd, rgbd_geo, rgb_geo


def gen_model_parts():
    """Outputs and gradients of the reference's own torchvision-free model code."""
    rgbd, rgbd_geo, rgb_geo = _load_models()
    out = {}
    # --- CrossModalAttention (pose_net_rgbd.py:8-35), eval mode (dropout off) ------
    # weights from a documented generator (xattn_weights, regenerated by the tests and
    # checked against the stored checksum) instead of 64 MB of fixture
    for name, (B, D, heads) in {"xattn": (2, 2048, 8), "xattn_small": (3, 64, 4)}.items():
        att = rgbd.CrossModalAttention(D, num_heads=heads, dropout=0.1).eval()
        sd = xattn_weights(D, seed=D + heads)
        att.load_state_dict(sd)
        g = torch.Generator().manual_seed(B * 100 + D)
        r = (torch.randn(B, D, generator=g)).requires_grad_(True)
        d = (torch.randn(B, D, generator=g) * 0.7 + 0.1).requires_grad_(True)
        y = att(r, d)
        w = torch.randn(B, D, generator=g)
        (y * w).sum().backward()
        out[f"{name}/weights_checksum"] = np.asarray([float(v.numpy().astype(np.float64).sum())
                                                      for v in sd.values()], np.float64)
        out[f"{name}/heads"] = np.asarray(heads, np.int32)
        out[f"{name}/rgb_feat"], out[f"{name}/depth_feat"], out[f"{name}/dout"] = (r.detach().numpy(),
                                                                                 d.detach().numpy(), w.numpy())
        out[f"{name}/out"] = y.detach().numpy()
        out[f"{name}/grad_rgb"], out[f"{name}/grad_depth"] = r.grad.numpy(), d.grad.numpy()
        for k, p in att.named_parameters():
            gr = p.grad.numpy()
            # weight gradients: the first 16 rows and the norm of the whole (bias grads whole)
            out[f"{name}/grad/{k}"] = gr[:16] if gr.ndim == 2 else gr
            out[f"{name}/gradnorm/{k}"] = np.asarray(np.linalg.norm(gr.astype(np.float64)), np.float64)
    # --- PoseNetRGBDGeometric._compute_pinhole_translation (:56-85) -----------------
    # `self` is unused by the method: called unbound on the reference's own function
    pin = rgbd_geo.PoseNetRGBDGeometric._compute_pinhole_translation
    g = torch.Generator().manual_seed(21)
    B = 16
    # piecewise-constant 8x8 blocks (compact fixture): < 0.01, in range, > 2.0
    depth = torch.rand(B, 28, 28, generator=g) * 2.4 - 0.2
    depth[depth.abs() < 0.05] = 0.0
    depth = depth.repeat_interleave(8, 1).repeat_interleave(8, 2).contiguous()
    bbox = torch.rand(B, 2, generator=g) * 300 - 40               # incl. < 0 and > 223
    bbox[0] = torch.tensor([223.9, 223.999])
    bbox[1] = torch.tensor([0.0, -0.5])
    bbox[2] = torch.tensor([112.5, 57.25])
    depth[2, 57, 112] = 0.0                                        # the z > 0.01 branch at a sampled pixel
    depth[3, :, :] = 5.0                                           # clamp at 2.0
    depth[4, :, :] = 0.05                                          # clamp at 0.1
    Kb = torch.zeros(B, 3, 3)
    Kb[:, 0, 0] = torch.rand(B, generator=g) * 800 + 300
    Kb[:, 1, 1] = torch.rand(B, generator=g) * 800 + 300
    Kb[:, 0, 2] = torch.rand(B, generator=g) * 224
    Kb[:, 1, 2] = torch.rand(B, generator=g) * 224
    Kb[:, 2, 2] = 1.0
    out["pin_depth/depth_raw"], out["pin_depth/bbox"], out["pin_depth/K"] = depth.numpy(), bbox.numpy(), Kb.numpy()
    out["pin_depth/out_Kb"] = pin(None, depth, bbox, Kb).numpy()
    out["pin_depth/out_K2"] = pin(None, depth, bbox, Kb[5]).numpy()     # a single (3, 3) K, expanded
    # --- PoseNetRGBGeometric._compute_pinhole_translation (:93-109), with grad ---------
    pinz = rgb_geo.PoseNetRGBGeometric._compute_pinhole_translation
    z = (torch.randn(B, 1, generator=g) * 0.3 + 0.8).requires_grad_(True)
    bb = torch.rand(B, 2, generator=g) * 640 - 20
    t = pinz(None, z, bb, Kb)
    wt = torch.randn(B, 3, generator=g)
    (t * wt).sum().backward()
    out["pin_z/z"], out["pin_z/bbox"], out["pin_z/K"], out["pin_z/dout"] = (z.detach().numpy(), bb.numpy(),
                                                                           Kb.numpy(), wt.numpy())
    out["pin_z/out_Kb"], out["pin_z/grad_z"] = t.detach().numpy(), z.grad.numpy()
    out["pin_z/out_K2"] = pinz(None, z.detach(), bb, Kb[7]).numpy()
    np.savez_compressed(os.path.join(OUT, "model_parts.npz"), **out)


class _StandInResNet(torch.nn.Module):
    """Trunk stand-in for the model fixture: ResNet's child layout (conv1, bn1, relu,
    maxpool, layer1-4, avgpool, fc -- so `children()[:-1]` and the depth model's
    `.conv1` swap, pose_net_rgbd.py:52-61, work unchanged) built from plain torch
    layers, (B, C, 224, 224) -> (B, 2048, 1, 1).  It is NOT torchvision's ResNet50
    and none of its arithmetic is pinned: the fixture records the features it hands
    the reference's own code, and the tests feed those recorded features -- not a
    trunk -- to the oracle and to the drop-in modules."""

    def __init__(self):
        super().__init__()
        nn = torch.nn
        self.conv1 = nn.Conv2d(3, 64, kernel_size=7, stride=2, padding=3, bias=False)
        self.bn1 = nn.BatchNorm2d(64)
        self.relu = nn.ReLU(inplace=True)
        self.maxpool = nn.MaxPool2d(3, 2, 1)
        self.layer1 = nn.Sequential(nn.Conv2d(64, 256, 1, bias=False), nn.ReLU())
        self.layer2 = nn.Sequential(nn.Conv2d(256, 512, 1, stride=2, bias=False), nn.ReLU())
        self.layer3 = nn.Sequential(nn.Conv2d(512, 1024, 1, stride=2, bias=False), nn.ReLU())
        self.layer4 = nn.Sequential(nn.Conv2d(1024, 2048, 1, stride=2, bias=False), nn.ReLU())
        self.avgpool = nn.AdaptiveAvgPool2d(1)
        self.fc = nn.Linear(2048, 1000)


class _StandInModels(types.ModuleType):
    """`torchvision.models` for the fixture run: resnet50(weights=None) -> _StandInResNet;
    ResNet50_Weights.DEFAULT exists only so the `pretrained` expression evaluates
    (the fixture constructs every model with pretrained=False)."""

    def __init__(self, name):
        super().__init__(name)
        self.ResNet50_Weights = types.SimpleNamespace(DEFAULT="IMAGENET1K_V2 (never loaded)")

    @staticmethod
    def resnet50(weights=None):
        if weights is not None:
            raise RuntimeError("the fixture never loads pretrained weights")
        return _StandInResNet()


def _load_models_standin():
    tv = types.ModuleType("torchvision")
    tvm = _StandInModels("torchvision.models")
    tv.models = tvm
    saved = {k: sys.modules.get(k) for k in ("torchvision", "torchvision.models")}
    sys.modules["torchvision"], sys.modules["torchvision.models"] = tv, tvm
    try:
        mods = {"PoseNetRGB": _load("ref_sm_rgb", "models/pose_net_rgb.py").PoseNetRGB,
                "PoseNetRGBGeometric": _load("ref_sm_rgb_geo", "models/pose_net_rgb_geometric.py").PoseNetRGBGeometric,
                "PoseNetRGBD": _load("ref_sm_rgbd", "models/pose_net_rgbd.py").PoseNetRGBD,
                "PoseNetRGBDGeometric": _load("ref_sm_rgbd_geo",
                                              "models/pose_net_rgbd_geometric.py").PoseNetRGBDGeometric}
    finally:
        for k, v in saved.items():
            if v is None:
                sys.modules.pop(k, None)
            else:
                sys.modules[k] = v
    return mods


# model -> (trunk attributes, forward argument names)
MODEL_SPECS = {
    "PoseNetRGB": (("backbone",), ("rgb",)),
    "PoseNetRGBGeometric": (("rgb_backbone",), ("rgb", "bbox", "K")),
    "PoseNetRGBD": (("rgb_backbone", "depth_backbone"), ("rgb", "depth")),
    "PoseNetRGBDGeometric": (("backbone",), ("rgb", "depth", "depth_raw", "bbox", "K")),
}
MODEL_B = 8
MODEL_INPUT_SEED = 4242
MODEL_WEIGHT_SEED = {"PoseNetRGB": 101, "PoseNetRGBGeometric": 102, "PoseNetRGBD": 103, "PoseNetRGBDGeometric": 104}
GRAD_ROWS = 4


def _record_grads(out, key, named):
    for k, p in named:
        if p.grad is None:
            continue
        g = p.grad.detach().numpy()
        out[f"{key}/grad/{k}"] = g[:GRAD_ROWS] if g.ndim >= 2 else g
        out[f"{key}/gradnorm/{k}"] = np.asarray(np.linalg.norm(g.astype(np.float64)), np.float64)
        out[f"{key}/gradsum/{k}"] = np.asarray(g.astype(np.float64).sum(), np.float64)


def gen_models(ref_pl):
    """The reference's four PoseNet classes run end to end with the trunk stand-in:
    every reference-owned layer around the trunk (heads, BN1d / LayerNorm MLPs, the
    normalisations incl. q/(||q||+1e-8), the z-CNN + z-MLP, CrossModalAttention +
    LN/GELU fusion, the pinholes) in eval mode and in train mode (Dropout modules
    in eval, BN with batch statistics), plus PoseLoss(1, 10) and its backward.
    Recorded: the trunk features, outputs, loss, feature gradients, parameter
    gradients (first rows, norm, sum), BN running statistics after the step, the
    z-CNN features; and the reference's own init constants (translation / z biases,
    xavier statistics of PoseNetRGBD's MLPs)."""
    from tests.synth import head_weights, model_inputs, tensor_checksum
    classes = _load_models_standin()
    inp = model_inputs(MODEL_B, MODEL_INPUT_SEED)
    out = {}
    for k, v in inp.items():
        out[f"inputs/checksum/{k}"] = np.asarray(tensor_checksum(v), np.float64)
    for k in ("bbox", "K", "gt_rot", "gt_trans"):
        out[f"inputs/{k}"] = inp[k].numpy()
    for name, (trunks, argnames) in MODEL_SPECS.items():
        # --- init constants of the reference's own constructor --------------------------
        torch.manual_seed(0)
        fresh = classes[name](pretrained=False)
        if hasattr(fresh, "trans_head"):
            out[f"{name}/init/trans_bias"] = fresh.trans_head[-1].bias.detach().numpy().copy()
        if hasattr(fresh, "z_predictor"):
            out[f"{name}/init/z_bias"] = fresh.z_predictor[-1].bias.detach().numpy().copy()
        if name == "PoseNetRGBD":
            for seqn in ("fusion", "rot_head", "trans_head"):
                for i, layer in enumerate(getattr(fresh, seqn)):
                    if isinstance(layer, torch.nn.Linear):
                        w = layer.weight.detach().double()
                        out[f"{name}/init/{seqn}.{i}/absmax_std"] = np.asarray([w.abs().max().item(),
                                                                                w.std().item()], np.float64)
                        out[f"{name}/init/{seqn}.{i}/bias_absmax"] = np.asarray(layer.bias.abs().max().item())
        # --- seeded parameters for everything outside the trunks -----------------------
        torch.manual_seed(1)
        m = classes[name](pretrained=False)
        shapes = {k: tuple(v.shape) for k, v in m.state_dict().items()}
        sd = head_weights(shapes, MODEL_WEIGHT_SEED[name])
        missing, unexpected = m.load_state_dict(sd, strict=False)
        assert not unexpected and all(k.startswith(("backbone.", "rgb_backbone.", "depth_backbone."))
                                      or k.endswith("num_batches_tracked") for k in missing), missing
        out[f"{name}/weights_checksum"] = np.asarray([tensor_checksum(sd[k]) for k in sorted(sd)], np.float64)
        feats = {}

        def hook(tn):
            def fn(mod, args, y):
                feats[tn] = y
                if y.requires_grad:
                    y.retain_grad()
            return fn
        handles = [getattr(m, tn).register_forward_hook(hook(tn)) for tn in trunks]
        zf = {}
        if name == "PoseNetRGBGeometric":
            def zhook(mod, args, y):
                zf["z"] = y
                if y.requires_grad:
                    y.retain_grad()
            handles.append(m.z_backbone.register_forward_hook(zhook))
        args = [inp[a] for a in argnames]
        # eval mode (running statistics, dropout off)
        m.eval()
        with torch.no_grad():
            rot, trans = m(*args)
        out[f"{name}/eval/rot"], out[f"{name}/eval/trans"] = rot.numpy(), trans.numpy()
        for tn in trunks:
            out[f"{name}/eval/feat/{tn}"] = feats[tn].reshape(MODEL_B, -1).numpy()
        if zf:
            out[f"{name}/eval/zfeat"] = zf["z"].numpy()
        # train mode, Dropout modules in eval, PoseLoss(1, 10)
        m.train()
        for mod in m.modules():
            if isinstance(mod, torch.nn.Dropout):
                mod.eval()
        rot, trans = m(*args)
        loss = ref_pl.PoseLoss(rot_weight=1.0, trans_weight=10.0, rotation_loss="geodesic")(
            rot, trans, inp["gt_rot"], inp["gt_trans"])
        loss.backward()
        out[f"{name}/train/rot"], out[f"{name}/train/trans"] = rot.detach().numpy(), trans.detach().numpy()
        out[f"{name}/train/loss"] = np.asarray(loss.item(), np.float64)
        for tn in trunks:
            out[f"{name}/train/feat/{tn}"] = feats[tn].detach().reshape(MODEL_B, -1).numpy()
            out[f"{name}/train/feat_grad/{tn}"] = feats[tn].grad.reshape(MODEL_B, -1).numpy()
        if zf:
            out[f"{name}/train/zfeat"] = zf["z"].detach().numpy()
            out[f"{name}/train/zfeat_grad"] = zf["z"].grad.numpy()
        _record_grads(out, f"{name}/train", [(k, p) for k, p in m.named_parameters()
                                             if not k.startswith(("backbone.", "rgb_backbone.", "depth_backbone."))])
        for k, v in m.state_dict().items():
            if k.startswith(("backbone.", "rgb_backbone.", "depth_backbone.")):
                continue
            if "running" in k or k.endswith("num_batches_tracked"):
                out[f"{name}/train/state/{k}"] = v.numpy().copy()
        for h in handles:
            h.remove()
    np.savez_compressed(os.path.join(OUT, "models.npz"), **out)


def main():
    os.makedirs(OUT, exist_ok=True)
    torch.set_num_threads(1)
    ref_pl = _load("ref_pose_loss", "models/pose_loss.py")
    ref_al = _load("ref_add_loss", "models/add_loss.py")
    only = sys.argv[1:]
    if not only or "pose_loss" in only:
        gen_pose_loss(ref_pl)
    if not only or "add" in only:
        gen_add(ref_al)
    if not only or "parts" in only:
        gen_model_parts()
    if not only or "models" in only:
        gen_models(ref_pl)
    for f in sorted(os.listdir(OUT)):
        print(f, os.path.getsize(os.path.join(OUT, f)))


if __name__ == "__main__":
    main()
