"""Host-issue and GPU-busy profile of the drop-in fp32 training path (the one the
reference's unchanged train_rgbd_geometric.py:106-112 runs: autograd through the drop-in
PoseNetRGBDGeometric, torch clip_grad_norm_, torch.optim.AdamW), bs32.

  python tools/dropin_profile.py [--steps N]            wall and host-issue ms per step
  rocprofv3 --kernel-trace -d D -o run -- python3 tools/dropin_profile.py --markers
  python tools/dropin_profile.py --analyze D            GPU-busy ms per step from the trace
(markers: a pose6d_pinhole_z_fwd launch, which this step never issues, before and after
the timed steps)."""
import argparse
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "6d-pose-estimation_amd")]


def analyze(d, steps):
    import glob
    import sqlite3
    db = glob.glob(os.path.join(d, "**", "*.db"), recursive=True)[0]
    rows = sqlite3.connect(db).execute("select name, start, end from kernels order by start").fetchall()
    marks = [i for i, r in enumerate(rows) if "pinhole_z_fwd" in r[0]]
    seg = rows[marks[0] + 1:marks[-1]]
    busy = sum(e - s for _, s, e in seg) / 1e6
    wall = (rows[marks[-1]][1] - rows[marks[0]][2]) / 1e6
    ours = sum(e - s for n, s, e in seg if "at::" not in n and "elementwise" not in n and "reduce" not in n.lower()
               or "wgrad_reduce" in n) / 1e6
    print(f"kernel trace, {steps} steps between markers: {len(seg) / steps:.0f} kernels/step, GPU busy "
          f"{busy / steps:.3f} ms/step of {wall / steps:.3f} ms wall ({100 * busy / wall:.1f} %); "
          f"pose6d kernels {ours / steps:.3f} ms/step, torch kernels (clip/AdamW/autograd glue) "
          f"{(busy - ours) / steps:.3f} ms/step")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--markers", action="store_true")
    ap.add_argument("--analyze", default="")
    a = ap.parse_args()
    if a.analyze:
        return analyze(a.analyze, a.steps)
    import torch
    from bench import synth_batch
    from models.pose_loss import PoseLoss
    from models.pose_net_rgbd_geometric import PoseNetRGBDGeometric
    from tools.step_profile import marker
    dev = torch.device("cuda")
    torch.manual_seed(0)
    model = PoseNetRGBDGeometric(pretrained=False).to(dev).train()
    opt = torch.optim.AdamW(model.parameters(), lr=1e-4, weight_decay=1e-4)
    crit = PoseLoss(rot_weight=1.0, trans_weight=10.0, rotation_loss="geodesic")
    rgb, depth_raw, bbox, K, gr, gt = synth_batch(32, dev, seed=7)

    def one():
        opt.zero_grad()
        rot, trans = model(rgb, None, depth_raw, bbox, K)
        loss = crit(rot, trans, gr, gt)
        loss.backward()
        torch.nn.utils.clip_grad_norm_(model.parameters(), 1.0)
        opt.step()
    for _ in range(3):
        one()
    torch.cuda.synchronize()
    if a.markers:
        marker()
    t0 = time.perf_counter()
    c0 = time.process_time()
    for _ in range(a.steps):
        one()
    t_issue = time.perf_counter() - t0
    c_issue = time.process_time() - c0
    if a.markers:
        marker()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    print(f"drop-in fp32 step: wall {wall / a.steps * 1e3:.3f} ms/step; host issue (loop returns) "
          f"{t_issue / a.steps * 1e3:.3f} ms/step, host CPU {c_issue / a.steps * 1e3:.3f} ms/step")


if __name__ == "__main__":
    main()
