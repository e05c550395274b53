"""Do independent branches of a captured hipGraph run concurrently on MI355X?
Two chains of small-grid kernels captured (a) on one stream, (b) forked onto two
streams; replay time of each.  Used to decide whether the downsample branch of
a bottleneck's first block can hide behind the main branch."""
import time

import torch


def chain(x, w, n):
    for _ in range(n):
        x = torch.mm(x, w).tanh_()
    return x


def run(mode, n=64, size=256, reps=50):
    dev = torch.device("cuda")
    a = torch.randn(size, size, device=dev) * 0.05
    b = torch.randn(size, size, device=dev) * 0.05
    w = torch.randn(size, size, device=dev) * 0.05
    side = torch.cuda.Stream()
    g = torch.cuda.CUDAGraph()
    main = torch.cuda.current_stream()
    for _ in range(2):   # warm-up outside capture
        chain(a, w, 2); chain(b, w, 2)
    torch.cuda.synchronize()
    with torch.cuda.graph(g):
        if mode == "serial":
            chain(a, w, n); chain(b, w, n)
        elif mode == "one":
            chain(a, w, n)
        else:
            cur = torch.cuda.current_stream()
            side.wait_stream(cur)
            with torch.cuda.stream(side):
                chain(b, w, n)
            chain(a, w, n)
            cur.wait_stream(side)
    g.replay(); torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        g.replay()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps * 1e3


if __name__ == "__main__":
    for size in (256, 1024):
        r = {m: run(m, size=size) for m in ("one", "serial", "fork")}
        print(f"size {size}: " + "  ".join(f"{k} {v:.3f} ms" for k, v in r.items()), flush=True)
