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
