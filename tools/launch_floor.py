"""Per-launch floor of a replayed hipGraph on this box (calibration for the step's ~330 launches).

Captures N back-to-back launches of (a) a one-element torch add (an almost empty kernel) and
(b) the same add on a 32 MiB tensor after a 64 MiB write (dirty L2 ahead of every tiny kernel),
replays each graph and prints wall us per launch.  Run under `rocprofv3 --kernel-trace --stats`
to see the per-kernel durations the step trace reports for its finalize kernels.

usage: python tools/launch_floor.py [--n 300]
"""
import argparse
import time

import torch


def replay_us(g, reps=20):
    torch.cuda.synchronize()
    g.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        g.replay()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e6


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=300)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    tiny = torch.zeros(1, device=dev)
    big = torch.zeros(8 << 20, device=dev)          # 32 MiB
    s = torch.cuda.Stream()
    cases = {}
    with torch.cuda.stream(s):
        for _ in range(3):
            tiny.add_(1)
            big.add_(1)
        torch.cuda.synchronize()
        g1 = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g1, stream=s, capture_error_mode="thread_local"):
            for _ in range(a.n):
                tiny.add_(1)
        cases["tiny x%d" % a.n] = (g1, a.n)
        g2 = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g2, stream=s, capture_error_mode="thread_local"):
            for _ in range(a.n // 10):
                big.add_(1)
                for _ in range(9):
                    tiny.add_(1)
        cases["(32MiB add + 9 tiny) x%d" % (a.n // 10)] = (g2, a.n)
        g3 = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g3, stream=s, capture_error_mode="thread_local"):
            for _ in range(a.n // 10):
                big.add_(1)
        cases["32MiB add x%d" % (a.n // 10)] = (g3, a.n // 10)
    for name, (g, n) in cases.items():
        us = replay_us(g)
        print("%-30s %9.1f us per replay  %6.2f us per launch" % (name, us, us / n), flush=True)


if __name__ == "__main__":
    main()
