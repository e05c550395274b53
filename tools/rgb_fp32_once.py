"""Run BASELINE configs[1] (drop-in PoseNetRGB bs32 fp32 eval forward) a few times,
for a kernel trace: rocprofv3 --kernel-trace -- python3 tools/rgb_fp32_once.py"""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "6d-pose-estimation_amd")]

from models.pose_net_rgb import PoseNetRGB  # noqa: E402


def main():
    dev = torch.device("cuda")
    torch.manual_seed(0)
    m = PoseNetRGB(pretrained=False).to(dev).set_compute_dtype(torch.float32).eval()
    x = torch.randn(32, 3, 224, 224, device=dev)
    with torch.no_grad():
        for _ in range(int(sys.argv[1]) if len(sys.argv) > 1 else 5):
            m(x)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
