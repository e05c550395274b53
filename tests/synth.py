"""Seeded synthetic inputs shared by the golden generator, the tests and bench.py.

Shapes follow SURVEY.md §8(d): LineMOD-like meshes (metres), poses with
quaternions in [x, y, z, w] order (dataset_rgbd.py:192-193, add_loss.py:205).
"""
import os

import numpy as np

# zero-based LineMOD object ids: folders 01,02,04,05,06,08,09,10,11,12,13,14,15
LINEMOD_OBJ_IDS = [0, 1, 3, 4, 5, 7, 8, 9, 10, 11, 12, 13, 14]


def _ply_text(verts_mm, faces=None):
    lines = ["ply", "format ascii 1.0", f"element vertex {len(verts_mm)}",
             "property float x", "property float y", "property float z"]
    if faces is not None:
        lines += [f"element face {len(faces)}", "property list uchar int vertex_indices"]
    lines.append("end_header")
    lines += [f"{x:.6f} {y:.6f} {z:.6f}" for x, y, z in verts_mm]
    if faces is not None:
        lines += [f"3 {a} {b} {c}" for a, b, c in faces]
    return "\n".join(lines) + "\n"


def write_mesh_dir(d, n_vertices=700, seed=11):
    """Write obj_XX.ply (ASCII, millimetres) + models_info.yml into directory d.

    Exercises the reference loader's paths (add_loss.py:29-99): official diameters
    for most objects, the max-pairwise fallback (no yml entry, >10 points), the
    0.1 m default (<=10 points), outliers beyond 0.5 m, face lines that the
    reference's parser also reads as vertices, and an unparsable file name.
    """
    rng = np.random.default_rng(seed)
    info = []
    for oid in LINEMOD_OBJ_IDS:
        folder = oid + 1
        if oid == 13:
            verts = rng.standard_normal((6, 3)) * 40.0          # <=10 pts -> 0.1 default
        else:
            verts = rng.standard_normal((n_vertices, 3)) * 40.0
            verts[:3] += 900.0                                  # outliers, ||p|| > 0.5 m
        faces = rng.integers(0, 40, size=(20, 3)) if oid in (4, 9) else None
        with open(os.path.join(d, f"obj_{folder:02d}.ply"), "w") as f:
            f.write(_ply_text(verts, faces))
        if oid not in (12, 13):                                  # 12: pairwise fallback
            info.append(f"{folder}: {{diameter: {100.0 + 7.5 * oid:.4f}, min_x: -50.0}}")
    info.append("junk: {diameter: 1.0}")                        # int('junk') fails -> skipped
    with open(os.path.join(d, "models_info.yml"), "w") as f:
        f.write("\n".join(info) + "\n")
    with open(os.path.join(d, "readme.ply"), "w") as f:          # name without '_' -> skipped
        f.write(_ply_text(np.zeros((3, 3))))


def make_poses(rng, B, sigma_q=0.05, sigma_t=0.005):
    """gt = random unit quaternion, pred = gt perturbed."""
    gr = rng.standard_normal((B, 4))
    gr /= np.linalg.norm(gr, axis=1, keepdims=True)
    pr = gr + sigma_q * rng.standard_normal((B, 4))
    pr /= np.linalg.norm(pr, axis=1, keepdims=True)
    gt = rng.standard_normal((B, 3)) * 0.1 + np.array([0.0, 0.0, 0.8])
    pt = gt + sigma_t * rng.standard_normal((B, 3))
    return (pr.astype(np.float32), pt.astype(np.float32), gr.astype(np.float32), gt.astype(np.float32))


def grid_mesh(rng, n):
    """Integer-millimetre mesh with duplicated vertices: exact distance ties."""
    pts = rng.integers(-30, 31, size=(n, 3)).astype(np.float32) / 1000.0
    dup = rng.integers(0, n, size=n // 5)
    pts[rng.integers(0, n, size=n // 5)] = pts[dup]
    return pts.astype(np.float32)


def synthetic_meshes(n_points=2000, seed=0, n_obj=13):
    """C4: 13 meshes of N points ~ N(0, 0.04^2) m, diameters 0.1-0.2 m."""
    rng = np.random.default_rng(seed)
    pts = {oid: (rng.standard_normal((n_points, 3)) * 0.04).astype(np.float32) for oid in LINEMOD_OBJ_IDS[:n_obj]}
    diam = {oid: 0.1 + 0.1 * i / 12.0 for i, oid in enumerate(LINEMOD_OBJ_IDS[:n_obj])}
    return pts, diam


def write_linemod_tree(root, n_frames=100, H=120, W=160, seed=0):
    """A LineMOD_preprocessed/data-shaped tree (folder/{rgb,depth}/NNNN.png,
    gt.yml, info.yml) exercising every branch of the reference index
    (data/dataset_rgbd.py:31-82): a non-numeric folder, a folder without
    info.yml, one without depth/ (RGB keeps it, RGB-D skips it), frames missing
    from gt.yml or info.yml, annotations of other objects on a frame, a
    non-PNG file among the frames and a missing depth PNG (read as zeros).
    Returns {folder: {frame_id: (rgb, depth or None)}} of what was written."""
    import yaml
    from PIL import Image
    from scipy.spatial.transform import Rotation
    rng = np.random.default_rng(seed)
    written = {}
    os.makedirs(os.path.join(root, "notes"), exist_ok=True)
    for folder in ("01", "03", "04", "06"):
        base = os.path.join(root, folder)
        os.makedirs(os.path.join(base, "rgb"), exist_ok=True)
        if folder != "04":
            os.makedirs(os.path.join(base, "depth"), exist_ok=True)
        gts, infos, frames = {}, {}, {}
        for f in range(n_frames):
            rgb = rng.integers(0, 256, (H, W, 3), dtype=np.uint8)
            Image.fromarray(rgb).save(os.path.join(base, "rgb", f"{f:04d}.png"))
            depth = None
            if folder != "04" and f != 18:
                depth = rng.integers(300, 1600, (H, W)).astype(np.uint16)
                depth[rng.random((H, W)) < 0.05] = 0
                Image.fromarray(depth).save(os.path.join(base, "depth", f"{f:04d}.png"))
            frames[f] = (rgb, depth)
            w, h = (int(v) for v in rng.integers(20, 70, 2))
            x, y = int(rng.integers(-10, W - w + 10)), int(rng.integers(-10, H - h + 10))
            R = Rotation.from_quat(rng.standard_normal(4)).as_matrix()
            anno = {"cam_R_m2c": [float(v) for v in R.reshape(-1)],
                    "cam_t_m2c": [float(v) for v in rng.normal((0, 0, 800), 80, 3)],
                    "obj_bb": [x, y, w, h], "obj_id": int(folder)}
            other = dict(anno, obj_id=int(folder) % 15 + 1, obj_bb=[1, 2, 30, 30])
            if f != 28:
                gts[f] = [other, anno] if f % 7 == 0 else [anno]
            if f != 38:
                fx = float(rng.uniform(500, 600))
                infos[f] = {"cam_K": [fx, 0.0, W / 2 + 3.5, 0.0, fx + 1.0, H / 2 - 2.25, 0.0, 0.0, 1.0],
                            "depth_scale": 1.0}
        with open(os.path.join(base, "rgb", "thumbs.db"), "w") as fh:
            fh.write("x")
        with open(os.path.join(base, "gt.yml"), "w") as fh:
            yaml.safe_dump(gts, fh)
        if folder != "03":
            with open(os.path.join(base, "info.yml"), "w") as fh:
                yaml.safe_dump(infos, fh)
        written[folder] = frames
    return written


def xattn_weights(D, seed):
    """CrossModalAttention parameters from a seeded CPU generator (q, k, v, out
    projections: N(0, 1/D) weights, N(0, 0.01) biases), as the model_parts fixture
    (tools/gen_goldens.py) was made with; the fixture stores their checksums."""
    import torch
    g = torch.Generator().manual_seed(seed)
    sd = {}
    for n in ("q_proj", "k_proj", "v_proj", "out_proj"):
        sd[n + ".weight"] = torch.randn(D, D, generator=g) * D ** -0.5
        sd[n + ".bias"] = torch.randn(D, generator=g) * 0.1
    return sd


TRUNK_PREFIXES = ("backbone.", "rgb_backbone.", "depth_backbone.")


def head_weights(shapes, seed):
    """Parameters and BN/LN buffers of a PoseNet's reference-owned layers (every
    state_dict key outside the ResNet50 trunks) from a seeded CPU generator, in
    sorted key order: >= 2-D weights N(0, 1/fan_in), 1-D weights 1 + N(0, 0.1^2),
    biases N(0, 0.1^2), running_mean N(0, 0.1^2), running_var U[0.5, 1.5);
    num_batches_tracked is left alone.  `shapes`: {key: shape}.  The model fixture
    (tools/gen_goldens.py gen_models) was made with it; the fixture stores the
    checksums the tests compare against."""
    import torch
    g = torch.Generator().manual_seed(seed)
    sd = {}
    for k in sorted(shapes):
        if k.startswith(TRUNK_PREFIXES) or k.endswith("num_batches_tracked"):
            continue
        shp = tuple(shapes[k])
        if k.endswith("running_mean"):
            v = torch.randn(shp, generator=g) * 0.1
        elif k.endswith("running_var"):
            v = torch.rand(shp, generator=g) + 0.5
        elif len(shp) >= 2:
            fan_in = 1
            for s in shp[1:]:
                fan_in *= s
            v = torch.randn(shp, generator=g) * fan_in ** -0.5
        elif k.endswith(".weight"):
            v = 1.0 + torch.randn(shp, generator=g) * 0.1
        else:
            v = torch.randn(shp, generator=g) * 0.1
        sd[k] = v
    return sd


def model_inputs(B, seed):
    """Seeded CPU inputs of the model fixture: rgb N(0,1) (B,3,224,224), depth U[0,1)
    (B,1,224,224), depth_raw U[0.3,1.6) m with ~5 % zeros (B,224,224), bbox centre
    U[0,223)^2, K with fx, fy U[400,800), cx, cy U[80,144), unit gt quaternion,
    gt translation around (0, 0, 0.8) m."""
    import torch
    g = torch.Generator().manual_seed(seed)
    rgb = torch.randn(B, 3, 224, 224, generator=g)
    depth = torch.rand(B, 1, 224, 224, generator=g)
    depth_raw = torch.rand(B, 224, 224, generator=g) * 1.3 + 0.3
    depth_raw[torch.rand(B, 224, 224, generator=g) < 0.05] = 0.0
    bbox = torch.rand(B, 2, generator=g) * 223
    K = torch.zeros(B, 3, 3)
    K[:, 0, 0] = torch.rand(B, generator=g) * 400 + 400
    K[:, 1, 1] = torch.rand(B, generator=g) * 400 + 400
    K[:, 0, 2] = torch.rand(B, generator=g) * 64 + 80
    K[:, 1, 2] = torch.rand(B, generator=g) * 64 + 80
    K[:, 2, 2] = 1.0
    gt_rot = torch.nn.functional.normalize(torch.randn(B, 4, generator=g), dim=1)
    gt_trans = torch.randn(B, 3, generator=g) * 0.1 + torch.tensor([0.0, 0.0, 0.8])
    return {"rgb": rgb, "depth": depth, "depth_raw": depth_raw, "bbox": bbox, "K": K,
            "gt_rot": gt_rot, "gt_trans": gt_trans}


def tensor_checksum(t):
    """(sum, sum of squares) in fp64: detects a drifted generator stream."""
    a = t.detach().cpu().numpy().astype(np.float64).ravel()   # numpy: independent of torch's thread count
    return [float(a.sum()), float((a * a).sum())]
