"""Eval-forward graph (bs32 bf16, as eval_graph_once.py) with every conv launch issued
TWICE back to back (same operands; the second instance finds them in cache): a kernel
trace then shows, per conv, the in-graph duration with producer-fresh operands (first)
against the hot replay (second).  Diagnostic only -- the outputs are identical.
rocprofv3 --kernel-trace -- python3 tools/eval_dup_trace.py 10"""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "6d-pose-estimation_amd")]

import pose6d.trunk as trunk  # noqa: E402
from bench import synth_batch  # noqa: E402
from models.pose_net_rgbd_geometric import PoseNetRGBDGeometric  # noqa: E402

_call = trunk.call


def dup_call(name, *args):
    _call(name, *args)
    if name in ("conv2d_fwd_act", "conv2d_fwd") and os.environ.get("DUP", "1") == "1":
        _call(name, *args)


trunk.call = dup_call


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    dev = torch.device("cuda")
    torch.manual_seed(0)
    m = PoseNetRGBDGeometric(pretrained=False).to(dev).set_compute_dtype(torch.bfloat16).eval()
    b = synth_batch(32, dev, seed=1)
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
