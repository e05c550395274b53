"""Drop-in for the reference's models/add_loss.py (ADDLoss, add_loss.py:13-215).

Host side (unchanged semantics): PLY/models_info.yml loading with the same
global-np.random draws (add_loss.py:29-99), so a seeded run selects the same
mesh points.  Device side: the whole batch is evaluated by one pose6d_add_eval
call (ADD, ADD-S nearest-point with bit-exact first-index argmin, 0.1d test)
followed by ONE device->host copy, instead of a Python loop with three
.item() syncs per sample.
"""
import os

import numpy as np
import torch
import torch.nn as nn

from pose6d._lib import call, require_device, stream

# LineMOD symmetric objects (eggbox and glue)  -- add_loss.py:10
SYMMETRIC_OBJECT_IDS = {9, 10}


class _MeshTable:
    """Packed device copy of ADDLoss.points (+ per-slot diameter / symmetry)."""

    def __init__(self, points, diameters, device):
        slots = (max(points) + 1) if points else 0
        off = np.zeros(max(slots, 1), np.int32)
        npts = np.zeros(max(slots, 1), np.int32)
        sym = np.zeros(max(slots, 1), np.uint8)
        diam = np.full(max(slots, 1), 0.1, np.float64)
        chunks, cur = [], 0
        for oid in sorted(points):
            p = points[oid].detach().to("cpu", torch.float32).reshape(-1, 3)
            off[oid], npts[oid] = cur, p.shape[0]
            sym[oid] = 1 if oid in SYMMETRIC_OBJECT_IDS else 0
            diam[oid] = float(diameters.get(oid, 0.1))          # add_loss.py:175
            chunks.append(p)
            cur += p.shape[0]
        pts = torch.cat(chunks) if chunks else torch.zeros(1, 3)
        self.n_slots = slots
        self.max_npts = int(npts.max()) if slots else 0
        self.points = pts.contiguous().to(device)
        self.off = torch.from_numpy(off).to(device)
        self.npts = torch.from_numpy(npts).to(device)
        self.sym = torch.from_numpy(sym).to(device)
        self.diam = torch.from_numpy(diam).to(device)
        self.key = _table_key(points, diameters)


def _table_key(points, diameters):
    return tuple((k, v.data_ptr(), tuple(v.shape), v._version) for k, v in sorted(points.items())) + \
        tuple(sorted(diameters.items()))


class ADDLoss(nn.Module):
    """ADD, ADD-S (symmetric objects) and ADD-0.1d accuracy for 6D pose evaluation."""

    def __init__(self, model_dir, device, rot_weight=0.0, trans_weight=0.0):
        super().__init__()
        self.points = {}
        self.diameters = {}
        self.device = device
        self.rot_weight = rot_weight
        self.trans_weight = trans_weight
        self._table = None
        self._load_models(model_dir)

    # ---------------------------------------------------------------- host side
    def _load_models(self, model_dir):
        """add_loss.py:29-81."""
        models_info_path = os.path.join(model_dir, "models_info.yml")
        official = {}
        if os.path.exists(models_info_path):
            import yaml
            with open(models_info_path, "r") as f:
                info = yaml.safe_load(f)
            for key, data in info.items():
                try:
                    oid = int(key) - 1
                    if "diameter" in data:
                        official[oid] = data["diameter"] / 1000.0
                except Exception:
                    pass
        num_points = 500
        for ply in sorted(f for f in os.listdir(model_dir) if f.endswith(".ply")):
            try:
                oid = int(ply.split("_")[1].split(".")[0]) - 1
            except Exception:
                continue
            pts = self._load_ply(os.path.join(model_dir, ply)) / 1000.0
            pts = pts[np.linalg.norm(pts, axis=1) < 0.5]
            if oid in official:
                diameter = official[oid]
            elif pts.shape[0] > 10:
                sample = pts[np.random.choice(pts.shape[0], min(100, pts.shape[0]), replace=False)]
                diameter = np.max(np.linalg.norm(sample[:, None] - sample[None, :], axis=2))
            else:
                diameter = 0.1
            self.diameters[oid] = diameter
            if pts.shape[0] > num_points:
                pts = pts[np.random.choice(pts.shape[0], num_points, replace=False)]
            self.points[oid] = torch.from_numpy(pts.astype(np.float32)).to(self.device)

    def _load_ply(self, path):
        """ASCII PLY vertices (add_loss.py:83-99): every post-header line with >= 3 tokens."""
        verts, header_end = [], False
        with open(path, "r") as f:
            for line in f:
                if "end_header" in line:
                    header_end = True
                    continue
                if header_end:
                    vals = line.strip().split()
                    if len(vals) >= 3:
                        verts.append([float(vals[0]), float(vals[1]), float(vals[2])])
        return np.array(verts)

    # -------------------------------------------------------------- device side
    def _mesh_table(self, device):
        key = _table_key(self.points, self.diameters)
        if self._table is None or self._table.key != key or self._table.points.device != device:
            self._table = _MeshTable(self.points, self.diameters, device)
        return self._table

    def per_sample(self, pred_r, pred_t, gt_r, gt_t, obj_ids, want_points=False):
        """Run pose6d_add_eval; returns device tensors (add, adds, valid, correct[, min, argmin])."""
        require_device(pred_r, pred_t, gt_r, gt_t, obj_ids)
        dev = pred_r.device
        B = pred_r.shape[0]
        T = self._mesh_table(dev)
        f = lambda t: t.detach().to(torch.float32).contiguous()
        ids = obj_ids.detach().to(torch.int64).contiguous()
        mx = max(T.max_npts, 1)
        mind = torch.empty(B, mx, device=dev, dtype=torch.float32)
        amin = torch.empty(B, mx, device=dev, dtype=torch.int32) if want_points else None
        ptadd = torch.empty(B, mx, device=dev, dtype=torch.float32)
        add = torch.empty(B, device=dev, dtype=torch.float64)
        adds = torch.empty(B, device=dev, dtype=torch.float64)
        valid = torch.empty(B, device=dev, dtype=torch.int32)
        correct = torch.empty(B, device=dev, dtype=torch.int32)
        call("add_eval", f(pred_r), f(pred_t), f(gt_r), f(gt_t), ids, B, T.points, T.off, T.npts, T.sym, T.diam,
             T.n_slots, T.max_npts, mind, amin, ptadd, add, adds, valid, correct, stream())
        out = {"add": add, "adds": adds, "valid": valid, "correct": correct}
        if want_points:
            out["min"], out["argmin"] = mind, amin
        return out

    @torch.no_grad()
    def eval_metrics(self, pred_r, pred_t, gt_r, gt_t, obj_ids):
        """add_loss.py:156-201 -- same dict, same mean-of-samples arithmetic."""
        if pred_r.shape[0] == 0:
            return {"add_mean": 0, "add_s_mean": 0, "add_01d_acc": 0}
        s = self.per_sample(pred_r, pred_t, gt_r, gt_t, obj_ids)
        host = torch.stack([s["add"], s["adds"], s["valid"].double(), s["correct"].double()]).cpu().numpy()
        v = host[2] > 0
        add, adds, corr = host[0][v].tolist(), host[1][v].tolist(), host[3][v].tolist()
        return {
            "add_mean": np.mean(add) * 1000 if add else 0,
            "add_s_mean": np.mean(adds) * 1000 if adds else 0,
            "add_01d_acc": np.mean(corr) * 100 if corr else 0,
        }

    def forward(self, pred_r, pred_t, gt_r, gt_t, obj_ids):
        """add_loss.py:101-150: mean over known samples of ADD (ADD-S for symmetric
        objects).  Returned as a device scalar; no gradient."""
        if pred_r.shape[0] == 0:
            return torch.tensor(0.0, device=pred_r.device, requires_grad=True)
        s = self.per_sample(pred_r, pred_t, gt_r, gt_t, obj_ids)
        T = self._table
        ids = obj_ids.detach().to(torch.int64)
        known = (ids >= 0) & (ids < max(T.n_slots, 1))
        sym = torch.zeros_like(known)
        sym[known] = T.sym[ids[known]].bool()
        per = torch.where(sym, s["adds"], s["add"])
        v = s["valid"] > 0
        cnt = v.sum()
        tot = torch.where(v, per, torch.zeros_like(per)).sum()
        return torch.where(cnt > 0, tot / cnt.clamp_min(1), torch.zeros_like(tot)).to(torch.float32)

    def train_loss(self, pred_r, pred_t, gt_r, gt_t, obj_ids):
        """Alias for forward() (add_loss.py:152-154)."""
        return self.forward(pred_r, pred_t, gt_r, gt_t, obj_ids)
