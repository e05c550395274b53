"""Replay the bs32 (or argv[2]) bf16 eval-forward graph of PoseNetRGBDGeometric (bench.py's
forward_roofline_eval) N times, for a kernel trace:
rocprofv3 --kernel-trace --stats -- python3 tools/eval_graph_once.py 20"""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "6d-pose-estimation_amd")]

from bench import synth_batch  # noqa: E402
from models.pose_net_rgbd_geometric import PoseNetRGBDGeometric  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 32
    dev = torch.device("cuda")
    torch.manual_seed(0)
    m = PoseNetRGBDGeometric(pretrained=False).to(dev).set_compute_dtype(torch.bfloat16).eval()
    b = synth_batch(B, dev, seed=1)
    args = (b[0], None, b[1], b[2], b[3])
    with torch.no_grad():
        s = torch.cuda.Stream(device=dev)
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            m(*args)
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            m(*args)
        for _ in range(n):
            g.replay()
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
