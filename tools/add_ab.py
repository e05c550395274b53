"""A/B of the ADD/ADD-S points kernel variants (POSE6D_ADD_VARIANT, read once per
process): times pose6d_add_eval on BASELINE configs[3] (bs256 x 2000 pts x 13 objects)
and saves min / argmin so the variants can be compared bit for bit.
usage: POSE6D_ADD_VARIANT=k python tools/add_ab.py OUT.npz"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "6d-pose-estimation_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from models.add_loss import ADDLoss  # noqa: E402
from tests.synth import LINEMOD_OBJ_IDS, make_poses, synthetic_meshes  # noqa: E402


def main():
    dev = torch.device("cuda")
    B, N = 256, 2000
    pts, diam = synthetic_meshes(N, seed=0)
    crit = ADDLoss.__new__(ADDLoss)
    torch.nn.Module.__init__(crit)
    crit.points = {k: torch.from_numpy(v).to(dev) for k, v in pts.items()}
    crit.diameters, crit.device, crit._table = diam, dev, None
    rng = np.random.default_rng(0)
    ids = np.array([LINEMOD_OBJ_IDS[i % len(LINEMOD_OBJ_IDS)] for i in range(B)], np.int64)
    args = [torch.from_numpy(a).to(dev) for a in (*make_poses(rng, B), ids)]
    out = crit.per_sample(*args, want_points=True)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts = []
    for _ in range(5):
        e0.record()
        for _ in range(10):
            crit.per_sample(*args)
        e1.record()
        e1.synchronize()
        ts.append(e0.elapsed_time(e1) / 10)
    ms = sorted(ts)[2]
    pairs = float(sum(pts[int(i)].shape[0] ** 2 for i in ids))
    print(f"variant {os.environ.get('POSE6D_ADD_VARIANT', '0')}: {ms:.4f} ms/batch, {pairs / ms / 1e9:.3f} T pairs/s, "
          f"{pairs * 8 / ms / 1e9 / 157.3:.3f} of 157.3 TF", flush=True)
    np.savez(sys.argv[1], min=out["min"].cpu().numpy(), argmin=out["argmin"].cpu().numpy(),
             adds=out["adds"].cpu().numpy())


if __name__ == "__main__":
    main()
