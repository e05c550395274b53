"""Graph-replayed BatchNorm finalize launches alone (calibration: what a finalize costs
beyond the ~1.5 us per-launch floor of an empty kernel, tools/launch_floor.py).

For each step shape (rows = ceil(M / 32) statistics rows, C channels): 50 back-to-back
pose6d_bn_finalize launches (the same partials: L2-warm after the first) vs 50 launches
alternating with a 16 MiB write (the partials' lines then come from HBM / another XCD, as
in the step) and 50 tiny torch adds; prints us per launch.

usage: python tools/fin_bench.py"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "6d-pose-estimation_amd")]

import torch  # noqa: E402

from pose6d._lib import call  # noqa: E402


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
    dev = torch.device("cuda")
    s = torch.cuda.Stream()
    big = torch.zeros(4 << 20, device=dev)
    tiny = torch.zeros(1, device=dev)
    N = 50
    for M, C in ((32 * 7 * 7, 512), (32 * 14 * 14, 256), (32 * 28 * 28, 128), (32 * 56 * 56, 64), (32 * 56 * 56, 256)):
        rows = (M + 31) // 32
        part = torch.rand(2, C, rows, device=dev) + 0.5
        part[0] *= 32
        g_ = torch.ones(C, device=dev)
        b_ = torch.zeros(C, device=dev)
        rm, rv = torch.zeros(C, device=dev), torch.ones(C, device=dev)
        outs = [torch.empty(C, device=dev) for _ in range(4)]

        def fin():
            call("bn_finalize", part, rows, C, M, g_, b_, rm, rv, None, 0.1, 1e-5, 1, *outs, None,
                 torch.cuda.current_stream().cuda_stream)

        res = {}
        with torch.cuda.stream(s):
            for _ in range(3):
                fin()
                big.add_(1)
                tiny.add_(1)
            torch.cuda.synchronize()
            for name, body, n in (("finalize x%d" % N, lambda: [fin() for _ in range(N)], N),
                                  ("(16MiB add + finalize) x%d" % N, lambda: [(big.add_(1), fin()) for _ in range(N)], N),
                                  ("16MiB add x%d" % N, lambda: [big.add_(1) for _ in range(N)], N),
                                  ("tiny add x%d" % N, lambda: [tiny.add_(1) for _ in range(N)], N)):
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, stream=s, capture_error_mode="thread_local"):
                    body()
                res[name] = replay_us(g) / n
        fin_cold = res["(16MiB add + finalize) x%d" % N] - res["16MiB add x%d" % N]
        print(f"M={M:6d} C={C:4d} rows={rows:5d}: finalize {res['finalize x%d' % N]:5.2f} us warm, "
              f"{fin_cold:5.2f} us after a 16 MiB write; tiny add {res['tiny add x%d' % N]:5.2f} us", flush=True)


if __name__ == "__main__":
    main()
