#!/usr/bin/env python3
"""Benchmark: crops/s of PoseNetRGBDGeometric training at batch 32 x 224^2 per GPU
(BASELINE.json metric; config 3 on one GPU, config 5 = the same per rank over
N GPUs).  A step = forward + PoseLoss(1, 10, geodesic) + backward +
clip_grad_norm_(1.0) + AdamW, the body of train_rgbd_geometric.py:97-115, on
synthetic device-resident inputs of the reference's shapes, bf16 trunk.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    (N > 1: python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N)

Prints ONE JSON line on rank 0 (contract in the task statement), including
"roofline" for the dominant kernel (HIP events, grouped by kernel symbol) and
"cpu_baseline" (the oracle's torch-CPU fp32 restatement of the same step,
rank 0 only, bounded sample).
"""
import argparse
import json
import os
import sys
import time
import warnings

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [REPO, os.path.join(REPO, "6d-pose-estimation_amd")]
warnings.simplefilter("ignore")

import torch  # noqa: E402

PEAK_BF16_TFLOPS = 2500.0   # MI355X dense bf16 MFMA (MI355X_MICROARCH.md)
PEAK_HBM_GBS = 8000.0       # HBM3E spec
FWD_BYTES_PER_CROP = 58.45e6   # bf16 fused-ideal forward bytes / crop
FWD_BYTES_PER_CROP_F32 = 116.89e6   # the same forward in fp32
# MI355X fp32 vector peak: 64 flop/clk/SIMD, reached by unpacked v_fma_f32
# (a wave64 instruction every 2 cycles on a SIMD-32) and by v_pk_fma_f32 alike
# (MI355X_MICROARCH.md constants table)
PEAK_F32_VALU_TFLOPS = 157.3
PEAK_F32_MFMA_TFLOPS = 157.3   # MI355X fp32 MFMA peak = the vector rate (MI355X_MICROARCH.md)
# PoseNetRGB forward FLOPs per crop: ResNet50 trunk 8.175 G + the two
# 2048-2048-1024-512-{4,3} heads (13.64 M multiply-adds)
RGB_FWD_FLOPS_PER_CROP = 8.175e9 + 2 * 13_635_072
ADD_FLOPS_PER_PAIR = 8.0       # 3 sub, 1 mul, 2 fma per ADD-S pair
# The committed PMC passes (tools/pmc_round.sh + tools/pmc_summary.py: separate FETCH_SIZE /
# WRITE_SIZE / SQ_VALU_MFMA_BUSY_CYCLES runs, FETCH_SIZE doubled for gfx950) the roofline
# `traffic` field is read from: one explicit file per compute dtype, updated in the commit
# that adds a newer pass (never picked by file-name order).  --pmc-bf16 / --pmc-f32 override.
PMC_SUMMARY = {"bf16": "profiles/r06h_pmc.json", "f32": "profiles/r06h_f32_pmc.json"}


def synth_batch(B, dev, seed):
    """SURVEY.md §8(d) synthetic inputs (seeded), resident on the device."""
    g = torch.Generator().manual_seed(seed)
    rgb = torch.randn(B, 3, 224, 224, generator=g)
    depth_raw = torch.rand(B, 224, 224, generator=g) * 1.3 + 0.3
    depth_raw[torch.rand(B, 224, 224, generator=g) < 0.05] = 0.0
    bbox = torch.rand(B, 2, generator=g) * 223
    s = 224.0 / (torch.rand(B, generator=g) * 200 + 100)
    K = torch.zeros(B, 3, 3)
    K[:, 0, 0] = K[:, 1, 1] = 572.4 * s
    K[:, 0, 2] = torch.rand(B, generator=g) * 224
    K[:, 1, 2] = torch.rand(B, generator=g) * 224
    K[:, 2, 2] = 1.0
    gt_rot = torch.nn.functional.normalize(torch.randn(B, 4, generator=g), dim=1)
    gt_trans = torch.randn(B, 3, generator=g) * 0.1 + torch.tensor([0.0, 0.0, 0.8])
    return [t.to(dev).contiguous() for t in (rgb, depth_raw, bbox, K, gt_rot, gt_trans)]


def host_cpu():
    """(threads the CPU baselines use, CPU model, os.cpu_count()).  The GPU box's
    os.cpu_count() reports the whole machine while a job gets a share of it (the
    affinity mask / cgroup quota): the baselines use that share, not oversubscribed."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            n = min(n, max(1, int(int(q) / int(per))))
    except (OSError, ValueError):
        pass
    model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return n, model, os.cpu_count()


def _cpu_meta(threads, model, total, kind, sample, value, unit):
    return {"value": value, "unit": unit, "cores": threads, "kind": kind, "sample": sample, "cpu_model": model,
            "os_cpu_count": total}


def cpu_baseline(batch=32, steps=7):
    """The oracle (torch-CPU fp32 restatement, shown equal to the reference on the
    golden fixtures) doing the same training step on the host cores.  Each of `steps`
    timed steps is clocked on its own: `value` is the batch over the MEDIAN step time,
    with the fastest / slowest steps beside it (a shared host's load moves single
    steps by tens of percent)."""
    from oracle import pose_loss as OP
    from oracle import resnet as OR
    from models.pose_net_rgbd_geometric import PoseNetRGBDGeometric
    threads, model, total = host_cpu()
    torch.set_num_threads(threads)
    torch.manual_seed(0)
    m = PoseNetRGBDGeometric(pretrained=False)
    P = {k: v.clone() for k, v in m.state_dict().items()}
    params = [v.requires_grad_(True) for k, v in P.items() if v.is_floating_point() and "running" not in k]
    opt = torch.optim.AdamW(params, lr=1e-4, weight_decay=1e-4)
    rgb, depth_raw, bbox, K, gr, gt = synth_batch(batch, "cpu", 123)

    def one():
        opt.zero_grad()
        rot, trans = OR.forward_rgbd_geometric(P, rgb, None, depth_raw, bbox, K, True)
        loss = OP.pose_loss(rot, trans, gr, gt, 1.0, 10.0)
        loss.backward()
        torch.nn.utils.clip_grad_norm_(params, 1.0)
        opt.step()
    one()
    times = []
    for _ in range(steps):
        t0 = time.perf_counter()
        one()
        times.append(time.perf_counter() - t0)
    times.sort()
    med = times[len(times) // 2]
    out = _cpu_meta(threads, model, total, "port",
                    f"oracle torch-CPU fp32 train step (fwd+loss+bwd+clip+AdamW), batch {batch}, {steps} steps timed "
                    f"one by one after 1 warmup, {threads} threads; value = batch / median step", round(batch / med, 3),
                    "crops/s")
    out["spread"] = {"median": round(batch / med, 3), "min": round(batch / times[-1], 3),
                     "max": round(batch / times[0], 3), "step_s": [round(t, 4) for t in times]}
    return out


def cpu_baseline_c1(batch=4, iters=5):
    """BASELINE configs[0] (C1): PoseNetRGB forward + PoseLoss at batch 4 on the CPU
    (oracle torch-CPU fp32 restatement; train-mode BN, no_grad, as BASELINE.md §3)."""
    from oracle import pose_loss as OP
    from oracle import resnet as OR
    from models.pose_net_rgb import PoseNetRGB
    threads, model, total = host_cpu()
    torch.set_num_threads(threads)
    torch.manual_seed(0)
    P = {k: v.clone() for k, v in PoseNetRGB(pretrained=False).state_dict().items()}
    rgb, _, _, _, gr, gt = synth_batch(batch, "cpu", 5)
    with torch.no_grad():
        def one():
            rot, trans = OR.forward_rgb(P, rgb, True)
            OP.pose_loss(rot, trans, gr, gt, 1.0, 10.0)
        one()
        t0 = time.perf_counter()
        for _ in range(iters):
            one()
        dt = time.perf_counter() - t0
    return _cpu_meta(threads, model, total, "port", f"oracle torch-CPU fp32 PoseNetRGB forward + PoseLoss, batch {batch}, "
                     f"{iters} timed iterations after 1 warmup", round(batch * iters / dt, 2), "crops/s")


def cpu_baseline_add(pts, diam, args, n=32):
    """BASELINE configs[3] (C4) on the CPU: the reference's eval_metrics loop
    (torch-CPU per-sample ops, oracle.add_loss.eval_metrics_torch) over the first
    `n` samples of the same synthetic bs256 x 2000-point batch."""
    from oracle import add_loss as OA
    threads, model, total = host_cpu()
    torch.set_num_threads(threads)
    P = {k: torch.from_numpy(v) for k, v in pts.items()}
    cargs = [a[:n].cpu() for a in args]
    OA.eval_metrics_torch(P, diam, *[a[:2] for a in cargs])
    t0 = time.perf_counter()
    OA.eval_metrics_torch(P, diam, *cargs)
    dt = time.perf_counter() - t0
    return _cpu_meta(threads, model, total, "port", f"reference eval_metrics loop restated in torch-CPU ops "
                     f"(oracle.add_loss.eval_metrics_torch), first {n} of the bs256 x 2000-point samples",
                     round(n / dt, 2), "samples/s")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-kernel-profile", action="store_true")
    ap.add_argument("--eager", action="store_true", help="no hipGraph capture")
    ap.add_argument("--no-side", action="store_true", help="skip the configs[1] / configs[3] side measurements")
    ap.add_argument("--no-fp32", action="store_true", help="skip the fp32 (reference precision) training line")
    ap.add_argument("--pmc-bf16", default=None, help="PMC summary json for the bf16 roofline traffic")
    ap.add_argument("--pmc-f32", default=None, help="PMC summary json for the fp32 roofline traffic")
    args = ap.parse_args()
    if args.pmc_bf16:
        PMC_SUMMARY["bf16"] = args.pmc_bf16
    if args.pmc_f32:
        PMC_SUMMARY["f32"] = args.pmc_f32

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if os.environ.get("POSE6D_BENCH_SHARE_GPU"):
        local %= torch.cuda.device_count()   # rehearsal of the N > 1 path on a one-GPU box only
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    pg = None
    if world > 1:
        import torch.distributed as dist
        if os.environ.get("POSE6D_BENCH_SHARE_GPU"):
            dist.init_process_group("gloo")   # RCCL refuses two ranks on one device
        else:
            dist.init_process_group("nccl", device_id=dev)
        pg = dist.group.WORLD

    from models.pose_net_rgbd_geometric import PoseNetRGBDGeometric
    from pose6d.train import RGBDGeometricTrainer

    torch.manual_seed(0)   # same init on every rank (replicated parameters)
    model = PoseNetRGBDGeometric(pretrained=False).to(dev)
    B = args.batch
    tr = RGBDGeometricTrainer(model, B, dtype=torch.bfloat16, process_group=pg)
    data = synth_batch(B, dev, seed=1000 + rank)   # each rank its own shard
    if not args.eager:
        tr.capture(data)
    for _ in range(args.warmup):
        tr.step(data)

    def barrier():
        if world > 1:
            torch.distributed.barrier()
        torch.cuda.synchronize()

    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        tr.step(data)
    barrier()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], device=dev)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        el = t.item()
    loss = tr.loss.item()
    ms = el / args.steps * 1e3
    value = world * B * args.steps / el

    result = {
        "metric": "crops/sec training RGBD-Geometric bs32 224^2 (per GPU), fwd+geodesic/L1 loss+bwd+clip+AdamW",
        "value": round(value, 2), "unit": "crops/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(ms, 4), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "bf16",
        "dtype_note": "bf16 trunk activations / MFMA operands as BASELINE configs[2] names (fp32 accumulation, "
                      "BN statistics, heads, loss, AdamW): narrower than the reference's fp32 training; the "
                      "reference-precision step is the fp32_train line",
        "data": "synthetic (SURVEY.md §8d shapes, device-resident)",
        "config": {"workload": "PoseNetRGBDGeometric train step (BASELINE configs[2]; configs[4] at N>1)",
                   "model": "PoseNetRGBDGeometric (ResNet50 + BN-MLP rot head, pinhole translation)",
                   "global_batch": world * B, "per_gpu_batch": B, "crop": "224x224", "seq_len": None,
                   "parallelism": f"dp{world}", "loss": float(loss)},
    }
    # every graph here is captured in thread-local mode, so the in-step roofline also runs
    # under a live RCCL group (whose watchdog thread polls collective events meanwhile;
    # tests/rccl_worker.py); the fp32 / side / CPU lines are one-GPU figures: N = 1 only
    solo = world == 1
    if not solo:
        result["side_measurements"] = "N=1 only (fp32_train, side_configs, cpu_baseline); roofline on rank 0"
    if rank == 0 and not args.no_kernel_profile:
        try:
            result.update(kernel_profile(tr, data, ms, with_forward=solo))
        except Exception as e:  # noqa: BLE001 - report, do not lose the scaling line
            result["roofline"] = {"error": repr(e)}
    if rank == 0 and solo and not args.no_fp32:
        # the same step in the reference's fp32 arithmetic (this headline line is bf16,
        # BASELINE configs[2]: narrower than the reference's fp32 training)
        result["fp32_train"] = fp32_train(dev, args.steps, args.warmup, B)
    if rank == 0 and solo and not args.no_side:
        result["side_configs"] = {"configs[1]": rgb_fp32_forward(dev), "dropin_fp32_train": dropin_fp32_train(dev),
                                  "configs[3]": add_eval_throughput(dev, cpu=not args.no_cpu_baseline),
                                  "frame_crops": crop_throughput(dev), "inference_b1": inference_latency(dev)}
    if rank == 0 and solo and not args.no_cpu_baseline:
        try:
            result["cpu_baseline"] = cpu_baseline()
        except Exception as e:  # noqa: BLE001 - report, do not fail the bench line
            result["cpu_baseline"] = {"value": None, "error": repr(e)}
        try:
            result.setdefault("side_configs", {})["configs[0]"] = {
                "workload": "PoseNetRGB forward + PoseLoss, batch 4, 224^2, CPU (BASELINE configs[0])",
                "cpu_baseline": cpu_baseline_c1()}
        except Exception as e:  # noqa: BLE001
            result.setdefault("side_configs", {})["configs[0]"] = {"error": repr(e)}
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


def kernel_profile(tr, data, step_ms, peak_tflops=None, with_forward=True, reps=10):
    """Dominant kernel of the step (largest total in-step time among the conv
    kernels, whose algorithmic flops are known) -> roofline object, timed INSIDE the
    captured step (pose6d.steptime: an event node spliced before every kernel node of
    the step's graph -- same launches, arguments and cache state as the timed step),
    plus the per-symbol in-step breakdown and the forward-pass HBM roofline
    fractions (the north-star's 60 % target)."""
    from pose6d import steptime
    if peak_tflops is None:
        peak_tflops = PEAK_BF16_TFLOPS if tr.trunk.dtype == torch.bfloat16 else PEAK_F32_MFMA_TFLOPS
    # the instrumented replays run whole AdamW steps: keep the trainer's state as the
    # timed loop left it (weights, moments, step counter / hyper-parameters, dropout seed)
    snap = tr.snapshot()
    timer = steptime.StepTimer(lambda: tr.step_body(data), tr.dev)
    recs = timer.run(reps, plain_ms=step_ms)
    inst_ms = timer.total_ms
    timer.close()
    tr.restore(snap)
    torch.cuda.synchronize()
    agg = steptime.by_symbol(recs)
    conv = {k: v for k, v in agg.items() if v["flops_known"] and v["flops"] > 0}
    sym, a = max(conv.items(), key=lambda kv: kv[1]["time_us"])
    avg_t = a["time_us"] / a["launches"] * 1e-6
    achieved = a["flops"] / a["launches"] / avg_t / 1e12
    conv_total_ms = sum(v["time_us"] for v in conv.values()) * 1e-3
    busy_ms = sum(r["us"] for r in recs) * 1e-3
    pmc, tsrc = pmc_traffic(sym, "bf16" if tr.trunk.dtype == torch.bfloat16 else "f32")
    traffic = round(pmc["hbm_bytes_per_launch"]) if pmc else None
    # SQ_VALU_MFMA_BUSY_CYCLES summed over the chip's 1024 SIMDs; busy fraction at 2.4 GHz
    mfma_busy = (round(pmc["mfma_busy_cycles_per_launch"] / (avg_t * 2.4e9 * 1024), 4)
                 if pmc and "mfma_busy_cycles_per_launch" in pmc else None)
    # the roof that binds this kernel: the larger of its MFMA time floor (algorithmic
    # flops / dense peak) and its HBM time floor (algorithmic bytes / 8 TB/s)
    nbytes = a["bytes"] / a["launches"]
    t_mfma = a["flops"] / a["launches"] / (peak_tflops * 1e12)
    t_hbm = nbytes / (PEAK_HBM_GBS * 1e9)
    hbm_gbs = nbytes / avg_t / 1e9
    if t_hbm > t_mfma:
        roof = {"bound": "hbm", "achieved": round(hbm_gbs, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                "frac": round(hbm_gbs / PEAK_HBM_GBS, 4)}
    else:
        roof = {"bound": "mfma", "achieved": round(achieved, 2), "peak": peak_tflops, "unit": "TFLOP/s",
                "frac": round(achieved / peak_tflops, 4)}
    out = {
        "roofline": {**roof, "traffic": traffic, "traffic_unit": "bytes/launch",
                     "mfma": {"achieved": round(achieved, 2), "peak": peak_tflops, "unit": "TFLOP/s",
                              "frac": round(achieved / peak_tflops, 4), "floor_us": round(t_mfma * 1e6, 2)},
                     "hbm": {"achieved": round(hbm_gbs, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                             "frac": round(hbm_gbs / PEAK_HBM_GBS, 4), "floor_us": round(t_hbm * 1e6, 2)},
                     "algorithmic_bytes_per_launch": round(nbytes),
                     "traffic_source": tsrc, "mfma_busy": mfma_busy,
                     "kernel": sym, "launches_per_step": a["launches"],
                     "avg_launch_us": round(avg_t * 1e6, 2),
                     "algorithmic_flops_per_launch": a["flops"] / a["launches"],
                     "timing": "in-step: HIP event nodes spliced around every kernel node of the captured step "
                               f"graph (pose6d/steptime.py), mean over {reps} replays, minus the calibrated event-node "
                               f"overhead ({timer.overhead_us:.2f} us/node = (instrumented - plain step) / nodes)",
                     "avg_launch_us_raw_events": round(a["time_raw_us"] / a["launches"], 2),
                     "per_launch": [[r["geom"], round(r["us"], 2),
                                     round(r["flops"] / (r["us"] * 1e-6) / 1e12, 1) if r["us"] > 0 else None,
                                     round((r.get("bytes") or 0) / (r["us"] * 1e-6) / 1e9, 1) if r["us"] > 0 else None]
                                    for r in recs if r["kernel"] == sym]},
        "breakdown": {"kernels_per_step": len(recs), "gpu_busy_ms_per_step": round(busy_ms, 3),
                      "instrumented_step_ms": round(inst_ms, 3), "step_ms": round(step_ms, 3),
                      "event_overhead_us_per_node": round(timer.overhead_us, 3),
                      "conv_kernels_ms_per_step": round(conv_total_ms, 3),
                      "by_symbol": {k: {"launches": v["launches"], "ms": round(v["time_us"] * 1e-3, 4),
                                        "avg_us": round(v["time_us"] / v["launches"], 2),
                                        **({"tflops": round(v["flops"] / (v["time_us"] * 1e-6) / 1e12, 1)}
                                           if v["flops_known"] and v["flops"] > 0 else {})}
                                    for k, v in agg.items()}},
    }
    if with_forward:
        # forward-only (training-mode BN) time of the trunk, graph-captured
        fwd_ms = forward_time(tr)
        fwd_gbs = FWD_BYTES_PER_CROP * tr.B / (fwd_ms * 1e-3) / 1e9
        # eval-mode forward of the whole model (BN folded into the conv epilogues), graph-captured
        ev_ms = eval_forward_time(tr.dev, tr.B)
        ev_gbs = FWD_BYTES_PER_CROP * tr.B / (ev_ms * 1e-3) / 1e9
        out["forward_roofline"] = {"bound": "hbm", "fwd_ms": round(fwd_ms, 4), "achieved": round(fwd_gbs, 1),
                                   "peak": PEAK_HBM_GBS, "unit": "GB/s", "frac": round(fwd_gbs / PEAK_HBM_GBS, 4),
                                   "algorithmic_bytes_per_crop": FWD_BYTES_PER_CROP,
                                   "mode": "trunk forward inside the training step (batch statistics)"}
        out["forward_roofline_eval"] = {"bound": "hbm", "fwd_ms": round(ev_ms, 4), "achieved": round(ev_gbs, 1),
                                        "peak": PEAK_HBM_GBS, "unit": "GB/s", "frac": round(ev_gbs / PEAK_HBM_GBS, 4),
                                        "algorithmic_bytes_per_crop": FWD_BYTES_PER_CROP,
                                        "crops_per_s": round(tr.B / (ev_ms * 1e-3), 1),
                                        "mode": "PoseNetRGBDGeometric eval forward bs32 bf16 (running-stat BN folded "
                                                "into the conv epilogues), hipGraph replay"}
    return out


def fp32_train(dev, steps, warmup, B=32):
    """The reference's own arithmetic (train_rgbd_geometric.py:106-112 trains in fp32,
    SURVEY.md §2.2): the fused RGBDGeometricTrainer step with fp32 activations and
    MFMA operands (exact v_mfma_f32_16x16x4_f32), graph-replayed at bs32, with its own
    in-step roofline against the fp32 MFMA peak."""
    from models.pose_net_rgbd_geometric import PoseNetRGBDGeometric
    from pose6d.train import RGBDGeometricTrainer
    torch.manual_seed(0)
    model = PoseNetRGBDGeometric(pretrained=False).to(dev)
    tr = RGBDGeometricTrainer(model, B, dtype=torch.float32)
    data = synth_batch(B, dev, seed=1000)
    tr.capture(data)
    for _ in range(warmup):
        tr.step(data)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        tr.step(data)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / steps * 1e3
    loss = float(tr.loss.item())   # read before the instrumented replays
    kp = kernel_profile(tr, data, ms, PEAK_F32_MFMA_TFLOPS, with_forward=False)
    return {"workload": "PoseNetRGBDGeometric train step, bs32 224^2, fp32 end to end (the reference's precision), "
                        "fused RGBDGeometricTrainer, hipGraph replay",
            "value": round(B / (ms * 1e-3), 2), "unit": "crops/s", "ms_per_step": round(ms, 4), "steps": steps,
            "dtype": "f32", "loss": loss, **kp}


def pmc_traffic(sym, dtype):
    """HBM bytes per launch of `sym` from the committed PMC summary named for this
    compute dtype in PMC_SUMMARY (made by tools/pmc_round.sh + tools/pmc_summary.py:
    separate FETCH_SIZE / WRITE_SIZE passes, FETCH_SIZE doubled for gfx950).  None when
    that file has no entry for the symbol (a kernel the pass predates)."""
    f = os.path.join(REPO, PMC_SUMMARY[dtype])
    try:
        k = json.load(open(f))["kernels"].get(sym)
    except (OSError, ValueError, KeyError):
        return None, PMC_SUMMARY[dtype]
    if k and "hbm_bytes_per_launch" in k:
        return k, PMC_SUMMARY[dtype]
    return None, PMC_SUMMARY[dtype]


def _time_fn(fn, reps):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / reps * 1e-3


def rgb_fp32_forward(dev, B=32, reps=10):
    """BASELINE configs[1]: PoseNetRGB bs32 224^2, fp32 (reference numerics), forward
    of the drop-in module (eval mode, no autograd) -> crops/s.  The fp32 forward is
    compute-bound (70 flop/B > the 19.7 flop/B fp32 ridge), so the
    roofline is the fp32 MFMA peak; the HBM fraction is kept beside it."""
    from models.pose_net_rgb import PoseNetRGB
    torch.manual_seed(0)
    m = PoseNetRGB(pretrained=False).to(dev).set_compute_dtype(torch.float32).eval()
    x = torch.randn(B, 3, 224, 224, device=dev)
    with torch.no_grad():
        t_eager = _time_fn(lambda: m(x), reps)
        # the same forward captured once into a hipGraph and replayed (as the eval
        # forward_roofline_eval line): the GPU-side rate without host launch gaps
        s = torch.cuda.Stream(device=dev)
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            m(x)
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, capture_error_mode="thread_local"):
            m(x)
        t = _time_fn(g.replay, reps)
    gbs = FWD_BYTES_PER_CROP_F32 * B / t / 1e9
    tf = RGB_FWD_FLOPS_PER_CROP * B / t / 1e12
    tf_eager = RGB_FWD_FLOPS_PER_CROP * B / t_eager / 1e12
    return {"workload": "PoseNetRGB forward, eval mode, bs32 224^2, fp32 (the drop-in module called eagerly, as the "
                        "reference's validation loop calls it; its hipGraph replay beside it)",
            "value": round(B / t_eager, 1), "unit": "crops/s", "ms_per_batch": round(t_eager * 1e3, 4),
            "graph_ms_per_batch": round(t * 1e3, 4), "graph_crops_per_s": round(B / t, 1), "dtype": "f32",
            "roofline": {"bound": "mfma", "achieved": round(tf_eager, 2), "peak": PEAK_F32_MFMA_TFLOPS,
                         "unit": "TFLOP/s", "frac": round(tf_eager / PEAK_F32_MFMA_TFLOPS, 4),
                         "frac_graph_replay": round(tf / PEAK_F32_MFMA_TFLOPS, 4),
                         "algorithmic_flops_per_crop": RGB_FWD_FLOPS_PER_CROP},
            "hbm_roofline": {"achieved": round(gbs, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                             "frac": round(gbs / PEAK_HBM_GBS, 4), "algorithmic_bytes_per_crop": FWD_BYTES_PER_CROP_F32}}


def dropin_fp32_train(dev, B=32, steps=5):
    """The path unchanged reference scripts run (train_rgbd_geometric.py:97-115): the
    drop-in PoseNetRGBDGeometric in its default fp32, driven by autograd, PoseLoss(1,
    10, geodesic), torch's clip_grad_norm_(1.0) and torch.optim.AdamW -- crops/s."""
    from models.pose_loss import PoseLoss
    from models.pose_net_rgbd_geometric import PoseNetRGBDGeometric
    torch.manual_seed(0)
    model = PoseNetRGBDGeometric(pretrained=False).to(dev).train()
    opt = torch.optim.AdamW(model.parameters(), lr=1e-4, weight_decay=1e-4)
    crit = PoseLoss(rot_weight=1.0, trans_weight=10.0, rotation_loss="geodesic")
    rgb, depth_raw, bbox, K, gr, gt = synth_batch(B, dev, seed=7)

    def one():
        opt.zero_grad()
        rot, trans = model(rgb, None, depth_raw, bbox, K)
        loss = crit(rot, trans, gr, gt)
        loss.backward()
        torch.nn.utils.clip_grad_norm_(model.parameters(), 1.0)
        opt.step()
        return loss
    for _ in range(2):
        one()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        one()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    return {"workload": "drop-in PoseNetRGBDGeometric fp32 train step through autograd + torch clip_grad_norm_ + "
                        "torch AdamW (train_rgbd_geometric.py:106-112 unchanged), bs32 224^2",
            "value": round(B / dt, 1), "unit": "crops/s", "ms_per_step": round(dt * 1e3, 3), "dtype": "f32"}


def add_eval_throughput(dev, B=256, N=2000, reps=10, cpu=True):
    """BASELINE configs[3]: ADD/ADD-S eval of bs256 x 2000 mesh points x 13 objects
    (SURVEY.md §8d synthetic meshes / perturbed poses) through ADDLoss.per_sample
    (one pose6d_add_eval call) -> samples/s, ADD-S pairs/s, fraction of the fp32
    vector peak at 8 flops per pair."""
    import numpy as np
    from models.add_loss import ADDLoss
    from tests.synth import LINEMOD_OBJ_IDS, make_poses, synthetic_meshes
    pts, diam = synthetic_meshes(N, seed=0)
    crit = ADDLoss.__new__(ADDLoss)
    torch.nn.Module.__init__(crit)
    crit.points = {k: torch.from_numpy(v).to(dev) for k, v in pts.items()}
    crit.diameters, crit.device, crit._table = diam, dev, None
    rng = np.random.default_rng(0)
    ids = np.array([LINEMOD_OBJ_IDS[i % len(LINEMOD_OBJ_IDS)] for i in range(B)], np.int64)
    args = [torch.from_numpy(a).to(dev) for a in (*make_poses(rng, B), ids)]
    t = _time_fn(lambda: crit.per_sample(*args), reps)
    pairs = float(sum(pts[int(i)].shape[0] ** 2 for i in ids))
    m = crit.eval_metrics(*args)
    extra = {}
    if cpu:
        try:
            extra["cpu_baseline"] = cpu_baseline_add(pts, diam, args)
        except Exception as e:  # noqa: BLE001
            extra["cpu_baseline"] = {"value": None, "error": repr(e)}
    return {**extra, "workload": f"ADDLoss eval bs{B} x {N} pts x {len(pts)} objects (ADD, ADD-S, 0.1d)",
            "value": round(B / t, 1), "unit": "samples/s", "ms_per_batch": round(t * 1e3, 4), "dtype": "f32",
            "pairs_per_s": round(pairs / t, 1), "add_01d_acc": round(float(m["add_01d_acc"]), 3),
            "valu_roofline": {"achieved": round(pairs * ADD_FLOPS_PER_PAIR / t / 1e12, 2),
                              "peak": PEAK_F32_VALU_TFLOPS, "peak_kind": "fp32 vector peak (v_fma_f32 / v_pk_fma_f32)",
                              "unit": "TFLOP/s",
                              "frac": round(pairs * ADD_FLOPS_PER_PAIR / t / 1e12 / PEAK_F32_VALU_TFLOPS, 4)}}


def crop_throughput(dev, B=32, reps=20):
    """North-star input path: 32 synthetic 640x480 frames (u8 RGB,
    u16 depth 300-1600 mm), bbox w, h ~ U[40, 200] inside the frame, jittered as in
    training -> pose6d_crop_rgbd (crop, pad, resize to 224, normalise, depth maps,
    crop-adjusted centre / K); timed separately from the model step.  HBM bytes:
    the source pixels the sampler touches (min(crop, 448)^2 clipped to the frame,
    3 + 2 B each) + 224^2 * 20 B written per crop."""
    import numpy as np
    from pose6d.data import CropRGBD, jitter_bboxes
    H, W, S = 480, 640, 224
    rng = np.random.default_rng(0)
    rgb = torch.from_numpy(rng.integers(0, 256, (B, H, W, 3), dtype=np.uint8)).to(dev)
    depth = torch.from_numpy(rng.integers(300, 1601, (B, H, W), dtype=np.uint16)).to(dev)
    w, h = rng.integers(40, 201, B), rng.integers(40, 201, B)
    bo = np.stack([rng.integers(0, W - w), rng.integers(0, H - h), w, h], 1).astype(np.int32)
    ba = jitter_bboxes(bo, True, np.random.RandomState(0))
    K = torch.tensor([[572.4114, 0, 325.2611], [0, 573.57043, 242.04899], [0, 0, 1]]).expand(B, 3, 3).contiguous()
    args = (rgb, depth, torch.from_numpy(bo).to(dev), torch.from_numpy(ba).to(dev), K.to(dev))
    crop = CropRGBD(S)
    out = crop(*args)
    t = _time_fn(lambda: crop(*args, out=out), reps)
    # the train transform (train_rgbd_geometric.py:41-47): + ColorJitter + RandomErasing
    from pose6d.data import TrainAugment
    crop_tr = CropRGBD(S, augment=TrainAugment(seed=0))
    crop_tr(*args, out=out)
    t_tr = _time_fn(lambda: crop_tr(*args, out=out), reps)
    nbytes = 0
    for x, y, ww, hh in ba.tolist():
        size = max(ww, hh) * 1.2
        n = int(size)
        x1, y1 = int(x + ww / 2 - size / 2), int(y + hh / 2 - size / 2)
        vis = max(0, min(W, x1 + n) - max(0, x1)) * max(0, min(H, y1 + n) - max(0, y1))
        nbytes += vis * min(1.0, (2 * S / n) ** 2) * 5 + S * S * 20
    gbs = nbytes / t / 1e9
    return {"workload": f"pose6d_crop_rgbd: {B} frames 640x480 -> 224^2 model inputs (val transform)",
            "value": round(B / t, 1), "unit": "crops/s", "ms_per_batch": round(t * 1e3, 4), "dtype": "u8/u16->f32",
            "train_transform": {"workload": "pose6d_crop_rgbd_train: the same crops + ColorJitter(0.3, 0.3, 0.3, "
                                            "0.05) + RandomErasing(0.2, (0.02, 0.1)) (train_rgbd_geometric.py:41-47)",
                                "value": round(B / t_tr, 1), "unit": "crops/s", "ms_per_batch": round(t_tr * 1e3, 4)},
            "hbm_roofline": {"achieved": round(gbs, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                             "frac": round(gbs / PEAK_HBM_GBS, 4), "algorithmic_bytes_per_batch": round(nbytes)}}


def inference_latency(dev, reps=50):
    """single-image inference (inference_*.py calls the model on one
    detected crop at a time): PoseNetRGBDGeometric eval forward at B=1, 224^2, with
    the pinhole translation -- latency per call, eager (one Python call of the drop-in
    module) and replayed from a captured hipGraph; fp32 (reference numerics) and bf16."""
    from models.pose_net_rgbd_geometric import PoseNetRGBDGeometric
    torch.manual_seed(0)
    out = {"workload": "PoseNetRGBDGeometric eval forward, B=1, 224^2 (+ pinhole translation)", "unit": "ms"}
    b = synth_batch(1, dev, seed=0)
    args = (b[0], None, b[1], b[2], b[3])
    for name, dt in (("f32", torch.float32), ("bf16", torch.bfloat16)):
        m = PoseNetRGBDGeometric(pretrained=False).to(dev).set_compute_dtype(dt).eval()
        with torch.no_grad():
            eager = _time_fn(lambda: m(*args), reps)
            s = torch.cuda.Stream(device=dev)
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                m(*args)
            torch.cuda.current_stream().wait_stream(s)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, capture_error_mode="thread_local"):
                m(*args)
            graph = _time_fn(g.replay, reps)
        out[name] = {"eager_ms": round(eager * 1e3, 4), "graph_ms": round(graph * 1e3, 4)}
    return out


def eval_forward_time(dev, B, reps=20):
    """PoseNetRGBDGeometric eval forward (rotation head + pinhole translation) of one
    bs-B batch in bf16, captured into a hipGraph; ms per replay."""
    from models.pose_net_rgbd_geometric import PoseNetRGBDGeometric
    torch.manual_seed(0)
    m = PoseNetRGBDGeometric(pretrained=False).to(dev).set_compute_dtype(torch.bfloat16).eval()
    b = synth_batch(B, dev, seed=1)
    args = (b[0], None, b[1], b[2], b[3])
    with torch.no_grad():
        s = torch.cuda.Stream(device=dev)
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            m(*args)
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, capture_error_mode="thread_local"):
            m(*args)
        return _time_fn(g.replay, reps) * 1e3


def forward_time(tr, reps=20):
    """Trunk + head forward of one batch (training-mode BN statistics), in a graph."""
    rgb = torch.randn(tr.B, 3, 224, 224, device=tr.dev)
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream(device=tr.dev)
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        tr.trunk.forward(rgb, True, pack=False)
    torch.cuda.current_stream().wait_stream(s)
    with torch.cuda.graph(g, capture_error_mode="thread_local"):
        tr.trunk.forward(rgb, True, pack=False)
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        g.replay()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / reps


if __name__ == "__main__":
    main()
