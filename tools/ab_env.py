"""A/B timing on one box: bs32 bf16 eval forward (hipGraph replay) and the bs32 bf16
training step, alternating between environment settings.
usage: python tools/ab_env.py VAR=A VAR=B [rounds]"""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "6d-pose-estimation_amd")]

import bench  # noqa: E402


def main():
    settings = [a.split("=", 1) for a in sys.argv[1:3]]
    rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    dev = torch.device("cuda")
    res = {i: [] for i in range(len(settings))}
    for r in range(rounds):
        for i, (k, v) in enumerate(settings):
            os.environ[k] = v
            res[i].append(bench.eval_forward_time(dev, 32, reps=50))
            print(f"round {r} {k}={v}: eval {res[i][-1]:.4f} ms", flush=True)
    for i, (k, v) in enumerate(settings):
        print(f"{k}={v}: eval min {min(res[i]):.4f} median {sorted(res[i])[len(res[i]) // 2]:.4f} ms")


if __name__ == "__main__":
    main()
