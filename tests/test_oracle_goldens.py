"""The oracle (CPU restatement) against golden vectors produced by the reference
itself (tools/gen_goldens.py).  CPU only."""
import json
import os
import tempfile

import numpy as np
import pytest
import torch

from oracle import add_loss as OA
from oracle import pose_loss as OP
from tests.synth import LINEMOD_OBJ_IDS, write_mesh_dir

HERE = os.path.dirname(os.path.abspath(__file__))


def test_pose_loss_matches_reference(golden):
    g = golden["pose_loss"]
    meta = json.load(open(os.path.join(HERE, "golden", "pose_loss.json")))
    for case in meta["cases"]:
        args = [g[f"{case}/{k}"] for k in ("pred_rot", "pred_trans", "gt_rot", "gt_trans")]
        for mode in meta["modes"]:
            kind, wr, wt = mode.split("_")
            loss, gr, gtr = OP.pose_loss_and_grads(*args, rot_weight=float(wr), trans_weight=float(wt),
                                                   rotation_loss=kind)
            key = f"{case}/{mode}"
            np.testing.assert_allclose(loss.numpy(), g[key + "/loss"], rtol=1e-6, atol=1e-7, err_msg=key)
            np.testing.assert_allclose(gr.numpy(), g[key + "/grad_rot"], rtol=1e-5, atol=1e-7, err_msg=key)
            np.testing.assert_allclose(gtr.numpy(), g[key + "/grad_trans"], rtol=1e-6, atol=0, err_msg=key)


def _points(g, tag):
    return {oid: g[f"{tag}/points/{oid}"] for oid in LINEMOD_OBJ_IDS if f"{tag}/points/{oid}" in g}


def _diams(g):
    return dict(zip(g["load/diam_ids"].tolist(), g["load/diam_vals"].tolist()))


@pytest.mark.parametrize("tag", ["n500", "n2000", "ties"])
def test_add_per_point_bit_exact(golden, tag):
    g = golden["add_loss"]
    pts = _points(g, "load" if tag == "n500" else tag)
    args = [g[f"{tag}/{k}"] for k in ("pred_rot", "pred_trans", "gt_rot", "gt_trans", "obj_ids")]
    s = OA.per_sample(pts, _diams(g), *args)
    np.testing.assert_array_equal(np.asarray(s["valid"]), g[f"{tag}/valid"])
    mins = np.concatenate(s["min"])
    amin = np.concatenate(s["argmin"])
    assert mins.tobytes() == g[f"{tag}/min_dist"].tobytes(), "ADD-S per-point min distance not bit-exact"
    np.testing.assert_array_equal(amin, g[f"{tag}/argmin"])
    np.testing.assert_allclose(s["add"], g[f"{tag}/add"], rtol=2e-6)
    np.testing.assert_allclose(s["adds"], g[f"{tag}/adds"], rtol=2e-6)
    m = OA.eval_metrics(pts, _diams(g), *args)
    ref = g[f"{tag}/metrics"]
    np.testing.assert_allclose([m["add_mean"], m["add_s_mean"], m["add_01d_acc"]], ref, rtol=2e-6)


def test_quat_to_mat_bit_exact(golden):
    g = golden["add_loss"]
    assert OA.quat_to_mat(g["n500/pred_rot"]).tobytes() == g["n500/pred_R"].tobytes()
    assert OA.quat_to_mat(g["n500/gt_rot"]).tobytes() == g["n500/gt_R"].tobytes()


def test_add_forward_and_edges(golden):
    g = golden["add_loss"]
    args = [g[f"n500/{k}"] for k in ("pred_rot", "pred_trans", "gt_rot", "gt_trans", "obj_ids")]
    np.testing.assert_allclose(OA.forward(_points(g, "load"), *args), g["n500/forward"], rtol=2e-6)
    m = OA.eval_metrics(_points(g, "load"), _diams(g), np.zeros((0, 4)), np.zeros((0, 3)), np.zeros((0, 4)),
                        np.zeros((0, 3)), np.zeros(0, np.int64))
    np.testing.assert_array_equal([m["add_mean"], m["add_s_mean"], m["add_01d_acc"]], g["empty/metrics"])


def test_loader_matches_reference(golden):
    g = golden["add_loss"]
    with tempfile.TemporaryDirectory() as d:
        write_mesh_dir(d, n_vertices=700, seed=11)
        np.random.seed(1234)
        pts, diam = OA.load_models(d)
    ref = _points(g, "load")
    assert sorted(pts) == sorted(ref)
    for oid in ref:
        assert pts[oid].tobytes() == ref[oid].tobytes(), oid
    assert sorted(diam) == g["load/diam_ids"].tolist()
    np.testing.assert_array_equal([diam[k] for k in sorted(diam)], g["load/diam_vals"])
