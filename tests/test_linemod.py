"""LineMOD evaluation harness (pose6d/linemod.py) on a
synthetic LineMOD tree (no LineMOD data or weights exist in the image, so the
ADD-0.1d target on real "cat" frames stays unmeasured).

CPU: the sample index against the rules of data/dataset_rgbd.py:31-82 and
dataset_rgb.py:31-78, the labels against scipy, the PNG decode, the per-object
filter and the mean-of-batch-means aggregation of compare_all_models.py:65-104.
GPU: each batch against the oracle's per-sample crop (oracle/crop.py) bit for
bit, and evaluate_model against the oracle ADD evaluation of the same
predictions."""
import os

import numpy as np
import pytest
import torch

from tests.synth import write_linemod_tree

N_FRAMES = 100


@pytest.fixture(scope="module")
def tree(tmp_path_factory):
    root = str(tmp_path_factory.mktemp("linemod"))
    return root, write_linemod_tree(root, n_frames=N_FRAMES)


def _expected(written, mode, rgbd):
    """(folder, frame) pairs the reference keeps, written out independently."""
    pick = {"val": 8, "test": 9}.get(mode)
    out = []
    for folder in ("01", "03", "04", "06"):
        if folder == "03" or (rgbd and folder == "04"):        # no info.yml / no depth dir
            continue
        for i in range(N_FRAMES):                              # sorted names == frame order here
            split_ok = (i % 10 == pick) if pick is not None else (i % 10 < 8)
            if split_ok and i not in (28, 38):                 # 28: not in gt.yml, 38: not in info.yml
                out.append((folder, i))
    return out


@pytest.mark.parametrize("mode", ["train", "val", "test"])
@pytest.mark.parametrize("rgbd", [True, False])
def test_index_follows_reference_rules(tree, mode, rgbd):
    from pose6d.linemod import LineMODSet
    root, written = tree
    ds = LineMODSet(root, mode, rgbd=rgbd)
    got = [(os.path.basename(os.path.dirname(os.path.dirname(it["img_path"]))),
            int(os.path.basename(it["img_path"])[:4])) for it in ds.all_data]
    assert got == _expected(written, mode, rgbd)
    assert all(it["obj_id"] == int(f) - 1 for (f, _), it in zip(got, ds.all_data))
    assert ds.augment_bbox == (mode == "train")
    assert all(("depth_path" in it) == rgbd for it in ds.all_data)


def test_object_filter(tree):
    from pose6d.linemod import CAT_FOLDER, LineMODSet
    root, written = tree
    a = LineMODSet(root, "val", objects=(CAT_FOLDER,))
    b = LineMODSet(root, "val", objects=(5,))
    assert [it["img_path"] for it in a.all_data] == [it["img_path"] for it in b.all_data]
    assert len(a) > 0 and all(it["obj_id"] == 5 for it in a.all_data)
    assert len(LineMODSet(root, "val", objects=("02",))) == 0
    with pytest.raises(FileNotFoundError):
        LineMODSet(os.path.join(root, "absent"), "val")


def test_labels_match_scipy_and_reference_casts(tree):
    from scipy.spatial.transform import Rotation
    from pose6d.linemod import LineMODSet
    root, _ = tree
    ds = LineMODSet(root, "val")
    q, t, ids = ds.labels(ds.all_data)
    for i, it in enumerate(ds.all_data):
        ref_q = torch.tensor(Rotation.from_matrix(np.array(it["cam_R_m2c"]).reshape(3, 3)).as_quat(),
                             dtype=torch.float32)
        assert torch.equal(q[i], ref_q)
        assert torch.equal(t[i], torch.tensor(np.array(it["cam_t_m2c"]), dtype=torch.float32) / 1000.0)
    assert ids.dtype == torch.long and ids.tolist() == [it["obj_id"] for it in ds.all_data]


def test_png_decode_round_trip(tree):
    from pose6d.linemod import load_depth, load_rgb
    root, written = tree
    rgb, depth = written["06"][8]
    assert np.array_equal(load_rgb(os.path.join(root, "06", "rgb", "0008.png")), rgb)
    d = load_depth(os.path.join(root, "06", "depth", "0008.png"), rgb.shape[:2])
    assert d.dtype == np.uint16 and np.array_equal(d, depth)
    missing = load_depth(os.path.join(root, "06", "depth", "0018.png"), rgb.shape[:2])
    assert missing.dtype == np.uint16 and not missing.any() and missing.shape == rgb.shape[:2]


def test_evaluate_model_mean_of_batch_means():
    """compare_all_models.py:92-104: the per-batch dict values are averaged with
    equal weight per batch (a short last batch counts as much as a full one)."""
    from pose6d.linemod import evaluate_model

    class Crit:
        def __init__(self):
            self.calls = 0

        def eval_metrics(self, pr, pt, gr, gt, ids):
            self.calls += 1
            n = float(pr.shape[0])
            return {"add_mean": n, "add_s_mean": 2 * n, "add_01d_acc": 100.0 / n}

    class Model(torch.nn.Module):
        def forward(self, rgb, *rest):
            self.nargs = 1 + len(rest)
            return torch.zeros(rgb.shape[0], 4), torch.zeros(rgb.shape[0], 3)

    z = lambda b, *s: torch.zeros(b, *s)
    batches = [(z(b, 3), z(b, 4), z(b, 3), torch.zeros(b, dtype=torch.long), z(b, 2), z(b, 3, 3)) for b in (16, 4)]
    m, crit = Model(), Crit()
    r = evaluate_model(m, "RGB-Geometric", batches, crit, is_rgbd=False, needs_geometry=True)
    assert crit.calls == 2 and m.nargs == 3 and not m.training
    assert r == {"ADD (mm)": 10.0, "ADD-S (mm)": 20.0, "ADD-0.1d (%)": (100 / 16 + 25) / 2}
    rgbd = [(z(b, 3), z(b, 1), z(b, 8, 8), z(b, 4), z(b, 3), torch.zeros(b, dtype=torch.long), z(b, 2), z(b, 3, 3))
            for b in (5,)]
    evaluate_model(m, "RGBD-Geometric", rgbd, crit, is_rgbd=True)
    assert m.nargs == 5
    evaluate_model(m, "RGBD", rgbd, crit, is_rgbd=True)
    assert m.nargs == 2
    assert evaluate_model(None, "RGB", batches, crit) is None


# ----------------------------------------------------------------- GPU
@pytest.mark.gpu
@pytest.mark.parametrize("rgbd", [True, False])
def test_batches_match_oracle_crop(tree, rgbd):
    from oracle import crop as OC
    from pose6d.linemod import LineMODSet
    root, written = tree
    ds = LineMODSet(root, "val", rgbd=rgbd)
    seen = 0
    for batch in ds.batches(6, "cuda"):
        torch.cuda.synchronize()
        b = [x.cpu() for x in batch]
        q, t, ids = ds.labels(ds.all_data[seen:seen + len(b[0])])
        for j in range(len(b[0])):
            it = ds.all_data[seen + j]
            folder = "%02d" % (it["obj_id"] + 1)
            rgb, depth = written[folder][int(os.path.basename(it["img_path"])[:4])]
            K = np.array(it["cam_K"], np.float32).reshape(3, 3)
            bb = np.array(it["bbox"], np.int32)
            d = depth if depth is not None else np.zeros(rgb.shape[:2], np.uint16)
            ref = OC.crop_sample(rgb, d if rgbd else None, bb, bb, K)
            if rgbd:
                got = [b[0][j], b[1][j], b[2][j], b[6][j], b[7][j]]
                for name, g, r in zip(("rgb", "depth", "depth_raw", "center", "K"), got, ref):
                    assert np.array_equal(g.numpy(), r), (seen + j, name)
                lab = b[3:6]
            else:
                assert np.array_equal(b[0][j].numpy(), ref[0]), seen + j
                x, y, w, h = it["bbox"]
                assert torch.equal(b[4][j], torch.tensor([x + w / 2, y + h / 2], dtype=torch.float32))
                assert torch.equal(b[5][j], torch.from_numpy(K))
                lab = b[1:4]
            assert torch.equal(lab[0][j], q[j]) and torch.equal(lab[1][j], t[j]) and lab[2][j] == ids[j]
        seen += len(b[0])
    assert seen == len(ds) == (16 if rgbd else 24)   # 8 val frames per kept folder; 6 + 6 + 4 (+ ...)


@pytest.mark.gpu
def test_evaluate_model_vs_oracle_add(tree, tmp_path):
    """The harness end to end on the GPU (model forward, ADDLoss.eval_metrics per
    batch) against the oracle's eval_metrics of the same predictions, averaged
    the same way."""
    from models.add_loss import ADDLoss
    from models.pose_net_rgbd_geometric import PoseNetRGBDGeometric
    from oracle import add_loss as OA
    from pose6d.linemod import LineMODSet, evaluate_model
    from tests.synth import write_mesh_dir
    root, _ = tree
    write_mesh_dir(str(tmp_path), n_vertices=300, seed=3)
    np.random.seed(7)
    crit = ADDLoss(str(tmp_path), "cuda")
    torch.manual_seed(0)
    model = PoseNetRGBDGeometric(pretrained=False).cuda().eval()
    ds = LineMODSet(root, "val")
    batches = list(ds.batches(6, "cuda"))      # 16 samples: 6 + 6 + 4, the short batch weighs the same
    got = evaluate_model(model, "RGBD-Geometric", batches, crit, is_rgbd=True)
    pts = {k: v.cpu().numpy() for k, v in crit.points.items()}
    ref = {"add": [], "adds": [], "acc": []}
    with torch.no_grad():
        for rgb, depth, depth_raw, gr, gt, ids, c, K in batches:
            pr, pt = model(rgb, depth, depth_raw, c, K)
            m = OA.eval_metrics(pts, crit.diameters, *(x.cpu().numpy() for x in (pr, pt, gr, gt, ids)))
            ref["add"].append(m["add_mean"])
            ref["adds"].append(m["add_s_mean"])
            ref["acc"].append(m["add_01d_acc"])
    np.testing.assert_allclose([got["ADD (mm)"], got["ADD-S (mm)"], got["ADD-0.1d (%)"]],
                               [np.mean(ref["add"]), np.mean(ref["adds"]), np.mean(ref["acc"])], rtol=1e-6)


@pytest.mark.gpu
def test_compare_models_cli_on_checkpoints(tree, tmp_path):
    """tools/compare_models.py end to end: reference-format checkpoints
    ({'model_state_dict': ...}, torch.save) of two models, cat-only filter."""
    import importlib.util
    from models.pose_net_rgb_geometric import PoseNetRGBGeometric
    from models.pose_net_rgbd_geometric import PoseNetRGBDGeometric
    from tests.synth import write_mesh_dir
    root, _ = tree
    write_mesh_dir(str(tmp_path), n_vertices=300, seed=3)
    torch.manual_seed(0)
    args = ["--data-root", root, "--model-dir", str(tmp_path), "--objects", "06", "--batch-size", "5"]
    for name, cls in (("RGB-Geometric", PoseNetRGBGeometric), ("RGBD-Geometric", PoseNetRGBDGeometric)):
        p = str(tmp_path / f"{name}.pth")
        torch.save({"epoch": 1, "model_state_dict": cls(pretrained=False).state_dict()}, p)
        args += ["--weights", f"{name}={p}"]
    args += ["--weights", f"RGB={tmp_path / 'absent.pth'}"]
    spec = importlib.util.spec_from_file_location(
        "compare_models", os.path.join(os.path.dirname(os.path.dirname(__file__)), "tools", "compare_models.py"))
    cm = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(cm)
    res = cm.main(args)
    assert sorted(res) == ["RGB-Geometric", "RGBD-Geometric"]
    for m in res.values():
        assert all(np.isfinite(v) for v in m.values())
        assert 0.0 <= m["ADD-0.1d (%)"] <= 100.0
