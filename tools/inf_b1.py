"""bench.py's B = 1 inference latency measurement alone (side_configs.inference_b1)."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "6d-pose-estimation_amd")]

import torch  # noqa: E402

import bench  # noqa: E402

r = bench.inference_latency(torch.device("cuda"))
print(os.environ.get("TAG", ""), json.dumps({k: r[k] for k in ("f32", "bf16")}), flush=True)
