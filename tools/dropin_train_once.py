"""Run N drop-in fp32 training steps (bench.py's dropin_fp32_train: autograd + torch
clip_grad_norm_ + torch AdamW around the drop-in PoseNetRGBDGeometric), for a kernel
trace: rocprofv3 --kernel-trace --stats -- python3 tools/dropin_train_once.py 6"""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "6d-pose-estimation_amd")]

from bench import synth_batch  # noqa: E402
from models.pose_loss import PoseLoss  # noqa: E402
from models.pose_net_rgbd_geometric import PoseNetRGBDGeometric  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    dev = torch.device("cuda")
    torch.manual_seed(0)
    model = PoseNetRGBDGeometric(pretrained=False).to(dev).train()
    opt = torch.optim.AdamW(model.parameters(), lr=1e-4, weight_decay=1e-4)
    crit = PoseLoss(rot_weight=1.0, trans_weight=10.0, rotation_loss="geodesic")
    rgb, depth_raw, bbox, K, gr, gt = synth_batch(32, dev, seed=7)
    for _ in range(n):
        opt.zero_grad()
        rot, trans = model(rgb, None, depth_raw, bbox, K)
        loss = crit(rot, trans, gr, gt)
        loss.backward()
        torch.nn.utils.clip_grad_norm_(model.parameters(), 1.0)
        opt.step()
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
