"""Host issue time vs GPU time of the training step, per path:
world 1 eager (~390 launches from Python), world 1 graph (one replay), and the
data-parallel step -- eager bucketed backward vs graph segments cut at bucket
boundaries with the all-reduces issued between replays.  Launch with
torch.distributed.run --nproc-per-node 2 and POSE6D_BENCH_SHARE_GPU=1 (both
ranks on one GPU over gloo: a rehearsal of the N > 1 host path; RCCL needs a GPU
per rank).  Prints one JSON line per rank.
"""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "6d-pose-estimation_amd")]

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def timed(fn, n):
    torch.cuda.synchronize()
    if dist.is_initialized():
        dist.barrier()
    t0 = time.perf_counter()
    host = 0.0
    for _ in range(n):
        h0 = time.perf_counter()
        fn()
        host += time.perf_counter() - h0
    torch.cuda.synchronize()
    return host / n * 1e3, (time.perf_counter() - t0) / n * 1e3


def main():
    from bench import synth_batch
    from models.pose_net_rgbd_geometric import PoseNetRGBDGeometric
    from pose6d.train import RGBDGeometricTrainer
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    pg = None
    if world > 1:
        dist.init_process_group("gloo")
        pg = dist.group.WORLD
    data = synth_batch(32, dev, seed=1000 + rank)
    out = {"rank": rank, "world": world}
    torch.manual_seed(0)
    tr = RGBDGeometricTrainer(PoseNetRGBDGeometric(pretrained=False).to(dev), 32, dtype=torch.bfloat16,
                              process_group=pg)
    for _ in range(2):
        tr.step_eager(data)
    out["eager_host_ms"], out["eager_wall_ms"] = timed(lambda: tr.step_eager(data), 10)
    tr.capture(data)
    for _ in range(2):
        tr.step()
    out["graph_host_ms"], out["graph_wall_ms"] = timed(tr.step, 20)
    out["graph_pieces"] = len(tr.graphs)
    out["buckets"] = len(tr.bucket_ends)
    print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
