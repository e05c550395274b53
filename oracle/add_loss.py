"""ORACLE — test infrastructure only.  Restatement of models/add_loss.py.

Per-point arithmetic runs in oracle/add_core.c (exact torch-CPU rounding);
the Python here restates the control flow of the reference's methods.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = os.path.join(HERE, "build", "liboracle_add.so")
SYMMETRIC_OBJECT_IDS = {9, 10}          # add_loss.py:10

_lib = None


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB):
            build()
        L = ctypes.CDLL(_LIB)
        P = ctypes.c_void_p
        I = ctypes.c_int64
        L.oracle_quat_to_mat.argtypes = [P, I, P]
        L.oracle_transform.argtypes = [P, I, P, P, P]
        L.oracle_add_dist.argtypes = [P, P, I, P]
        L.oracle_adds_min.argtypes = [P, P, I, P, P]
        _lib = L
    return _lib


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def quat_to_mat(q):
    """add_loss.py:203-215."""
    q = np.ascontiguousarray(q, np.float32)
    R = np.empty((q.shape[0], 3, 3), np.float32)
    lib().oracle_quat_to_mat(_p(q), q.shape[0], _p(R))
    return R


def transform(P, R, t):
    """add_loss.py:178-179: mm(P, R.T) + t."""
    P = np.ascontiguousarray(P, np.float32)
    R = np.ascontiguousarray(R, np.float32)
    t = np.ascontiguousarray(t, np.float32)
    out = np.empty_like(P)
    lib().oracle_transform(_p(P), P.shape[0], _p(R), _p(t), _p(out))
    return out


def add_dist(Pp, G):
    Pp, G = np.ascontiguousarray(Pp, np.float32), np.ascontiguousarray(G, np.float32)
    d = np.empty(Pp.shape[0], np.float32)
    lib().oracle_add_dist(_p(Pp), _p(G), Pp.shape[0], _p(d))
    return d


def adds_min(Pp, G):
    Pp, G = np.ascontiguousarray(Pp, np.float32), np.ascontiguousarray(G, np.float32)
    n = Pp.shape[0]
    d = np.empty(n, np.float32)
    i = np.empty(n, np.int32)
    lib().oracle_adds_min(_p(Pp), _p(G), n, _p(d), _p(i))
    return d, i


def per_sample(points, diameters, pred_r, pred_t, gt_r, gt_t, obj_ids):
    """add_loss.py:159-195 without the final averaging.  Returns, for the valid
    samples only (oid in points), ADD, ADD-S, correct flag, per-point min
    distances and argmins (lists), plus the validity mask over the batch."""
    pR, gR = quat_to_mat(pred_r), quat_to_mat(gt_r)
    out = {"add": [], "adds": [], "correct": [], "min": [], "argmin": [], "valid": []}
    for i in range(len(obj_ids)):
        oid = int(obj_ids[i])
        if oid not in points:                       # add_loss.py:171-172
            out["valid"].append(0)
            continue
        out["valid"].append(1)
        P = points[oid]
        G = transform(P, gR[i], gt_t[i])
        Q = transform(P, pR[i], pred_t[i])
        add = float(np.mean(add_dist(Q, G), dtype=np.float64))
        m, j = adds_min(Q, G)
        adds = float(np.mean(m, dtype=np.float64))
        thr = 0.1 * diameters.get(oid, 0.1)          # add_loss.py:175-176
        eff = adds if oid in SYMMETRIC_OBJECT_IDS else add
        out["add"].append(add)
        out["adds"].append(adds)
        out["correct"].append(1.0 if eff < thr else 0.0)
        out["min"].append(m)
        out["argmin"].append(j)
    return out


def eval_metrics(points, diameters, pred_r, pred_t, gt_r, gt_t, obj_ids):
    """add_loss.py:156-201."""
    s = per_sample(points, diameters, pred_r, pred_t, gt_r, gt_t, obj_ids)
    return {
        "add_mean": np.mean(s["add"]) * 1000 if s["add"] else 0,
        "add_s_mean": np.mean(s["adds"]) * 1000 if s["adds"] else 0,
        "add_01d_acc": np.mean(s["correct"]) * 100 if s["correct"] else 0,
    }


def forward(points, pred_r, pred_t, gt_r, gt_t, obj_ids):
    """add_loss.py:101-150 (grouped ADD / ADD-S loss), accumulated in float64."""
    pR, gR = quat_to_mat(pred_r), quat_to_mat(gt_r)
    total, count = 0.0, 0
    for i in range(len(obj_ids)):
        oid = int(obj_ids[i])
        if oid not in points:
            continue
        P = points[oid]
        G = transform(P, gR[i], gt_t[i])
        Q = transform(P, pR[i], pred_t[i])
        if oid in SYMMETRIC_OBJECT_IDS:
            total += float(np.mean(adds_min(Q, G)[0], dtype=np.float64))
        else:
            total += float(np.mean(add_dist(Q, G), dtype=np.float64))
        count += 1
    return 0.0 if count == 0 else total / count


def forward_torch(points, pred_r, pred_t, gt_r, gt_t, obj_ids):
    """add_loss.py:101-150 restated with torch ops (differentiable: the gradient
    reference for pose6d_add_loss_bwd).  points: dict oid -> (N, 3) fp32 tensor;
    groups by object in first-appearance order as the reference does."""
    import torch

    def q2m(q):   # add_loss.py:203-215
        x, y, z, w = q[:, 0], q[:, 1], q[:, 2], q[:, 3]
        x2, y2, z2 = x * x, y * y, z * z
        xy, xz, yz = x * y, x * z, y * z
        wx, wy, wz = w * x, w * y, w * z
        r0 = torch.stack([1 - 2 * y2 - 2 * z2, 2 * xy - 2 * wz, 2 * xz + 2 * wy], dim=1)
        r1 = torch.stack([2 * xy + 2 * wz, 1 - 2 * x2 - 2 * z2, 2 * yz - 2 * wx], dim=1)
        r2 = torch.stack([2 * xz - 2 * wy, 2 * yz + 2 * wx, 1 - 2 * x2 - 2 * y2], dim=1)
        return torch.stack([r0, r1, r2], dim=1)

    pR, gR = q2m(pred_r), q2m(gt_r)
    groups = {}
    for i in range(pred_r.shape[0]):
        oid = int(obj_ids[i])
        if oid in points:
            groups.setdefault(oid, []).append(i)
    total = torch.zeros((), dtype=pred_r.dtype)
    count = 0
    for oid, idx in groups.items():
        idx = torch.tensor(idx, dtype=torch.long)
        P = points[oid].to(pred_r.dtype)
        G = torch.matmul(P.unsqueeze(0), gR[idx].transpose(-1, -2)) + gt_t[idx].unsqueeze(1)
        Q = torch.matmul(P.unsqueeze(0), pR[idx].transpose(-1, -2)) + pred_t[idx].unsqueeze(1)
        if oid in SYMMETRIC_OBJECT_IDS:
            per = torch.norm(Q.unsqueeze(2) - G.unsqueeze(1), dim=3).min(dim=2)[0].mean(dim=1)
        else:
            per = torch.norm(Q - G, dim=2).mean(dim=1)
        total = total + per.sum()
        count += len(idx)
    return total / count if count else total


def load_models(model_dir, num_points=500):
    """add_loss.py:29-99 (loader), including its quirks: every post-header line
    with >= 3 tokens is a vertex, diameters from models_info.yml (mm -> m),
    max-pairwise fallback over <=100 random points, global np.random draws."""
    import yaml
    official = {}
    info = os.path.join(model_dir, "models_info.yml")
    if os.path.exists(info):
        with open(info) as f:
            mi = yaml.safe_load(f)
        for k, v in mi.items():
            try:
                oid = int(k) - 1
                if "diameter" in v:
                    official[oid] = v["diameter"] / 1000.0
            except Exception:
                pass
    points, diameters = {}, {}
    for fn in sorted(f for f in os.listdir(model_dir) if f.endswith(".ply")):
        try:
            oid = int(fn.split("_")[1].split(".")[0]) - 1
        except Exception:
            continue
        verts, header_end = [], False
        with open(os.path.join(model_dir, fn)) as f:
            for line in f:
                if "end_header" in line:
                    header_end = True
                    continue
                if header_end:
                    v = line.strip().split()
                    if len(v) >= 3:
                        verts.append([float(v[0]), float(v[1]), float(v[2])])
        pts = np.array(verts) / 1000.0
        pts = pts[np.linalg.norm(pts, axis=1) < 0.5]
        if oid in official:
            diam = official[oid]
        elif pts.shape[0] > 10:
            s = pts[np.random.choice(pts.shape[0], min(100, pts.shape[0]), replace=False)]
            diam = np.max(np.linalg.norm(s[:, None] - s[None, :], axis=2))
        else:
            diam = 0.1
        diameters[oid] = diam
        if pts.shape[0] > num_points:
            pts = pts[np.random.choice(pts.shape[0], num_points, replace=False)]
        points[oid] = pts.astype(np.float32)
    return points, diameters


def eval_metrics_torch(points, diameters, pred_r, pred_t, gt_r, gt_t, obj_ids):
    """add_loss.py:156-201 as the reference runs it: torch-CPU ops per sample
    (mm + t, norm, the (N, N, 3) pairwise tensor, min over the gt points) --
    the CPU baseline of BASELINE configs[3] (bench.py), on the host's threads.
    points: {oid: (N, 3) float32 torch tensor}; the rest torch tensors."""
    import torch

    def q2m(q):                                              # add_loss.py:203-215
        x, y, z, w = q[:, 0], q[:, 1], q[:, 2], q[:, 3]
        return torch.stack([
            torch.stack([1 - 2 * y * y - 2 * z * z, 2 * x * y - 2 * w * z, 2 * x * z + 2 * w * y], 1),
            torch.stack([2 * x * y + 2 * w * z, 1 - 2 * x * x - 2 * z * z, 2 * y * z - 2 * w * x], 1),
            torch.stack([2 * x * z - 2 * w * y, 2 * y * z + 2 * w * x, 1 - 2 * x * x - 2 * y * y], 1)], 1)

    pR, gR = q2m(pred_r), q2m(gt_r)
    adds_, addss, corr = [], [], []
    for i in range(pred_r.shape[0]):
        oid = int(obj_ids[i].item())
        if oid not in points:
            continue
        P = points[oid]
        G = torch.mm(P, gR[i].T) + gt_t[i]
        Q = torch.mm(P, pR[i].T) + pred_t[i]
        add = torch.norm(Q - G, dim=1, p=2).mean().item()
        adds = torch.norm(Q.unsqueeze(1) - G.unsqueeze(0), dim=2).min(dim=1)[0].mean().item()
        d = adds if oid in SYMMETRIC_OBJECT_IDS else add
        adds_.append(add)
        addss.append(adds)
        corr.append(float(d < 0.1 * diameters.get(oid, 0.1)))
    return {"add_mean": np.mean(adds_) * 1000 if adds_ else 0, "add_s_mean": np.mean(addss) * 1000 if addss else 0,
            "add_01d_acc": np.mean(corr) * 100 if corr else 0}
