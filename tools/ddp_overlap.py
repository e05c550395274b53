"""Predicted N-GPU overlap of the bucketed gradient all-reduce with the backward
(verdict r03 item 8; UNMEASURED on hardware: no 8-GPU node was available).

On one GPU: the bs32 training step is captured exactly as the world-1 trainer
captures it, with the trunk backward's on_conv_done hook (the point where the DDP
path issues a bucket, train.py _backward_ddp) recording the graph position; the
step is replayed with an event before every node (pose6d.steptime), which gives the
in-step time at which every 25 MB bucket's last producing kernel ends.  A model of
the comm stream then replays the buckets in order: bucket i starts at
max(ready_i, end_{i-1}) and takes  alpha + 2 (N-1)/N * bytes_i / busbw  (ring
all-reduce); the unhidden tail is the comm end minus the backward end, and the
predicted weak-scaling efficiency at N GPUs is step / (step + tail).  Compute slowed
by RCCL's own kernels (CUs and HBM it takes during the backward) is not modelled.

usage: python tools/ddp_overlap.py [--dtype bf16|f32] [--out profiles/r04_ddp_overlap.json]
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "6d-pose-estimation_amd")]

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "f32"])
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--bucket-mb", type=float, default=25.0)
    ap.add_argument("--tail-mb", default="0,2,4,8", help="last-bucket caps to model (0 = none; the trainer's "
                                                        "default is 2)")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    from bench import synth_batch
    from models.pose_net_rgbd_geometric import PoseNetRGBDGeometric
    from pose6d import steptime
    from pose6d.dist import plan_buckets
    from pose6d.train import RGBDGeometricTrainer

    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    dtype = torch.bfloat16 if a.dtype == "bf16" else torch.float32
    model = PoseNetRGBDGeometric(pretrained=False).to(dev)
    tr = RGBDGeometricTrainer(model, a.batch, dtype=dtype)
    data = synth_batch(a.batch, dev, seed=1000)
    # the DDP trainer's buckets (train.py: plan_buckets over the arena in gradient order)
    sizes = [(off, p.numel()) for p, off in zip(tr.arena.params, tr.arena.offsets)]
    plans = {}
    for t in [float(v) for v in a.tail_mb.split(",")]:
        ends = plan_buckets(sizes, int(a.bucket_mb * 1e6 / 4), int(t * 1e6 / 4))
        ends[-1] = (ends[-1][0], tr.arena.numel)
        plans[f"tail{t:g}MB"] = [e for _, e in ends]

    tr.capture(data)
    for _ in range(3):
        tr.step(data)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        tr.step(data)
    e1.record()
    e1.synchronize()
    step_ms = e0.elapsed_time(e1) / 20

    marks = []   # (graph nodes so far, arena prefix final)
    state = {"log": None, "bwd_start": None}

    def body():
        tr.trunk.pack_weights(force=True)
        tr._forward_loss(*data)
        dfeat = tr._head_backward()
        log = state["log"]
        state["bwd_start"] = log.node_count() if log else None

        def on_conv(op):
            last = op.conv.bias if op.conv.bias is not None else op.conv.weight
            if state["log"] is not None:
                marks.append((state["log"].node_count(), tr.arena.end_offset(last)))
        tr.trunk.backward(dfeat, tr.arena.grad_of, on_conv_done=on_conv)
        state["bwd_end"] = log.node_count() if log else None
        tr._optimizer()

    # StepTimer captures body() once (after a warm run); expose its call log to body()
    orig = steptime._CallLog

    class _Log(orig):
        def __init__(self, s):
            super().__init__(s)
            state["log"] = self

    steptime._CallLog = _Log
    snap = tr.snapshot()
    try:
        state["log"] = None
        timer = steptime.StepTimer(body, dev)
    finally:
        steptime._CallLog = orig
    recs = timer.run(a.reps, plain_ms=step_ms)
    n_nodes = len(timer.records)
    durs = [r["us"] for r in timer.records]   # every node (kernel and memset) in graph order
    timer.close()
    tr.restore(snap)
    cum = [0.0]
    for d in durs:
        cum.append(cum[-1] + d)
    step_us = cum[-1]
    bwd_start_us = cum[state["bwd_start"]]
    bwd_end_us = cum[state["bwd_end"]]

    def model(bucket_ends):
        # ready time of each bucket: the first mark whose prefix covers the bucket end
        ready = []
        for be in bucket_ends:
            t = None
            for nodes, upto in marks:
                if upto >= be:
                    t = cum[min(nodes, n_nodes)]
                    break
            ready.append(bwd_end_us if t is None else t)
        sizes_b = [4 * (e - s) for s, e in zip([0] + bucket_ends[:-1], bucket_ends)]
        scen = {}
        for N in (2, 4, 8):
            for name, busbw, alpha in (("one_link_153GBps", 153e9, 30.0), ("rccl_300GBps", 300e9, 30.0),
                                       ("rccl_500GBps", 500e9, 30.0)):
                t_end = 0.0
                starts = []
                for r, b in zip(ready, sizes_b):
                    t0 = max(r, t_end)
                    dur = alpha + 2 * (N - 1) / N * b / busbw * 1e6
                    t_end = t0 + dur
                    starts.append((round(t0, 1), round(dur, 1)))
                tail = max(0.0, t_end - bwd_end_us)
                scen[f"N{N}_{name}"] = {"tail_us": round(tail, 1),
                                        "comm_total_us": round(sum(d for _, d in starts), 1),
                                        "predicted_efficiency": round(step_us / (step_us + tail), 4),
                                        "buckets_start_dur_us": starts}
        return {"buckets": [{"bytes": b, "ready_us": round(r, 1)} for b, r in zip(sizes_b, ready)],
                "scenarios": scen}

    res = {"dtype": a.dtype, "batch_per_rank": a.batch, "bucket_mb": a.bucket_mb, "step_ms_plain": round(step_ms, 4),
           "step_us_instrumented_sum": round(step_us, 1), "backward_start_us": round(bwd_start_us, 1),
           "backward_end_us": round(bwd_end_us, 1), "gradient_bytes": 4 * tr.arena.numel,
           "model": "comm stream replays buckets in order: start = max(ready, previous end), duration = alpha + "
                    "2(N-1)/N * bytes / busbw; tail = comm end - backward end; efficiency = step / (step + tail); "
                    "UNMEASURED on hardware (no multi-GPU node); RCCL's compute interference not modelled; "
                    "plans: the 25 MB greedy buckets with the last bucket capped at tail MB (trainer default 2)",
           "plans": {k: model(v) for k, v in plans.items()}}
    print(json.dumps(res, indent=1))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
