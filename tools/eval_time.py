"""ms per bs32 bf16 eval forward (PoseNetRGBDGeometric, hipGraph replay) and per fp32
configs[1] forward, as one JSON line -- for build A/B timing (tools/ab_lib.sh ... eval)."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "6d-pose-estimation_amd")]

import torch  # noqa: E402

import bench  # noqa: E402

if __name__ == "__main__":
    dev = torch.device("cuda", 0)
    ms = bench.eval_forward_time(dev, 32, reps=50)
    print(json.dumps({"ms_per_step": round(ms, 4)}))
