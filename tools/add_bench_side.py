"""bench.py's configs[3] ADD measurement alone (same function, no CPU baseline)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "6d-pose-estimation_amd")]

import torch  # noqa: E402

import bench  # noqa: E402

r = bench.add_eval_throughput(torch.device("cuda"), cpu=False)
print(f"{os.environ.get('TAG', '')}: bench configs[3] {r['ms_per_batch']:.4f} ms/batch, VALU frac {r['valu_roofline']['frac']}",
      flush=True)
