"""Whole-step trainer for the north-star workload: PoseNetRGBDGeometric training
(forward + PoseLoss(1, 10, geodesic) + backward + clip_grad_norm_(1.0) + AdamW),
i.e. the per-batch body of the reference's train() loop
(scripts/training/train_rgbd_geometric.py:97-115), without autograd or host syncs.

MI355X design:
  * one flat fp32 arena for parameters / gradients / AdamW moments (the module's
    Parameters become views into it: state_dict, checkpoints, torch optimizers
    keep working), parameters laid out in gradient-completion order so that DDP
    buckets are contiguous prefixes that become ready one after another;
  * the entire step (~400 launches) is captured once into a hipGraph and
    replayed; the AdamW step counter, dropout seed and lr live in device memory
    so replays stay exact;
  * the AdamW launch also writes the convs' packed compute-dtype weights
    (pose6d_adamw_step_packed): the next forward reads them with no packing pass
    over the updated masters.  A write to the masters from outside the step that
    goes through the arena or a Parameter (restore, load_state_dict, an in-place op
    on a Parameter under no_grad) is seen through torch's version counters and
    re-packed before the next step.  A write through `p.data` (e.g.
    `p.data.copy_(w)`) is NOT seen -- `.data` is an alias with a version counter
    of its own -- so such a caller must call sync_weights() afterwards (as a
    torch user must re-run anything cached from the old values);
  * data parallel: one process per GPU, batch shards, gradient all-reduce over
    RCCL (torch.distributed 'nccl'); bucketed all-reduces are issued on a comm
    stream as soon as each bucket's gradients exist, overlapping the rest of the
    backward.  For that the captured step is cut into segments at the launches
    that complete a bucket: replay = segment, all-reduce of the buckets it
    finished (comm stream, event-ordered), next segment, ..., then the
    optimizer graph once every all-reduce has landed (a handful of host calls
    per step instead of ~300 eager launches).
"""
import math
import os

import numpy as np
import torch

from ._lib import Pose6dError, call, query, stream
from .dist import BucketReducer, plan_buckets
from .head import HeadEngine
from .trunk import TrunkEngine

NPART = 1024
# POSE6D_HEAD_WGRAD_SIDE=1: the head's Linear weight gradients on a side stream in the
# one-GPU step (step_body) -- bit-identical, but the replayed graph with that one parallel
# branch measured 0.35 ms SLOWER per step (bf16 4.48 -> 4.84 ms, fp32 11.58 -> 11.90 ms,
# profiles/r06h_head_side_stream_rejected.txt): off, kept for A/B
POSE6D_HEAD_WGRAD_SIDE = os.environ.get("POSE6D_HEAD_WGRAD_SIDE", "0") == "1"


class FlatArena:
    """Parameters (in the given order) re-homed into one flat fp32 buffer."""

    def __init__(self, params, device, align=64):
        self.params = list(params)
        self.offsets = []
        off = 0
        for p in self.params:
            self.offsets.append(off)
            off += (p.numel() + align - 1) // align * align
        self.numel = off
        self.flat = torch.zeros(off, device=device, dtype=torch.float32)
        self.grad = torch.zeros(off, device=device, dtype=torch.float32)
        self._views = {}
        with torch.no_grad():
            for p, o in zip(self.params, self.offsets):
                v = self.flat[o:o + p.numel()].view_as(p)
                v.copy_(p.data)
                p.data = v
                self._views[id(p)] = self.grad[o:o + p.numel()].view_as(p)

    def grad_of(self, p):
        return self._views[id(p)]

    def _index_of(self, p):
        if not hasattr(self, "_index"):
            self._index = {id(q): i for i, q in enumerate(self.params)}
        return self._index[id(p)]

    def end_offset(self, p):
        i = self._index_of(p)
        return self.offsets[i] + self.params[i].numel()


class RGBDGeometricTrainer:
    """Fused, graph-captured training step for PoseNetRGBDGeometric."""

    def __init__(self, model, batch, dtype=torch.bfloat16, lr=1e-4, weight_decay=1e-4, max_norm=1.0,
                 betas=(0.9, 0.999), eps=1e-8, rot_weight=1.0, trans_weight=10.0, process_group=None,
                 bucket_mb=25.0, tail_mb=2.0, force_buckets=False, pack_in_adamw=True):
        self.model = model
        self.B = batch
        dev = next(model.parameters()).device
        self.dev = dev
        model.train()
        self.trunk = TrunkEngine(model.backbone, 3)
        self.trunk.set_dtype(dtype)
        self.trunk.prepare(batch, 224, 224, dtype, dev)
        self.head = HeadEngine(model.rot_head)
        order = self.head.params_in_grad_order() + self.trunk.params_in_grad_order()
        assert len(order) == len(list(model.parameters())) and {id(p) for p in order} == \
            {id(p) for p in model.parameters()}
        self.arena = FlatArena(order, dev)
        self.m = torch.zeros_like(self.arena.flat)
        self.v = torch.zeros_like(self.arena.flat)
        # pack_in_adamw=False: the previous layout (a packing launch at the start of every
        # step, plain adamw_step) -- kept for A/B timing and the bit-identity test
        self.pack_in_adamw = pack_in_adamw
        self._packed_key = None
        self.sync_weights()
        if pack_in_adamw:
            self._build_jobs()
        self.world = torch.distributed.get_world_size(process_group) if process_group is not None else 1
        # the bucketed all-reduce path (segmented graphs, comm stream, async collectives):
        # every world > 1, and world 1 with force_buckets (exercises the RCCL branch on a
        # one-GPU box: an all-reduce over one rank returns its input)
        self._ddp = process_group is not None and (self.world > 1 or force_buckets)
        # hp[6]: gradient scale read by adamw_step -- 1/world averages the all-reduced sum
        # inside the update (exact for power-of-two world sizes: scaling by 2^-k commutes
        # with every rounding; arena.grad then holds the SUM after a step).  Other world
        # sizes average the all-reduced SUM in a pass of their own before the clip
        # (g_sum * (1/world), rounded once), and hp[6] stays 1.  That is a post-all-reduce
        # average: torch DDP's Reducer pre-scales each rank's gradient by 1/world before
        # the all-reduce, so for non-power-of-two worlds the two differ in the last bit.
        # The reference trains on one GPU (no DDP), so this rounding is parity unpinned.
        self._avg_pass = self.world > 1 and (self.world & (self.world - 1)) != 0
        scale = 1.0 if (self.world == 1 or self._avg_pass) else 1.0 / self.world
        self.hp = torch.tensor([lr, betas[0], betas[1], eps, weight_decay, 0.0, scale, max_norm],
                               device=dev, dtype=torch.float32)
        self.partials = torch.zeros(NPART, device=dev)
        self.norm = torch.zeros(1, device=dev)
        self.loss = torch.zeros((), device=dev)
        self.rot = torch.empty(batch, 4, device=dev)
        self.trans = torch.empty(batch, 3, device=dev)
        self.drot = torch.empty(batch, 4, device=dev)
        self.dtrans = torch.empty(batch, 3, device=dev)
        self.draw = torch.empty(batch, 4, device=dev)
        self.one = torch.ones((), device=dev)
        self.seed = torch.tensor([torch.initial_seed() & 0x7FFFFFFFFFFF], device=dev, dtype=torch.int64)
        self.wr, self.wt = float(rot_weight), float(trans_weight)
        self.pg = process_group
        self.graphs = None
        self._buckets(bucket_mb, tail_mb)

    # ------------------------------------------------------------- packed weights
    def _build_jobs(self):
        """The work table of pose6d_adamw_step_packed (plain ranges and 64 x 64 conv
        tiles over the arena), built once: the arena and the packed buffers never move."""
        rec = self.trunk._desc_host
        args = (rec.ctypes.data, len(rec), self.arena.flat.data_ptr(), self.arena.numel)
        n = query("adamw_packed_jobs", *args, None, 0)
        if n <= 0:
            raise Pose6dError(f"pose6d_adamw_packed_jobs failed ({n})")
        jobs = np.zeros((n, 4), dtype=np.int32)
        if query("adamw_packed_jobs", *args, jobs.ctypes.data, n) != n:
            raise Pose6dError("pose6d_adamw_packed_jobs: inconsistent job count")
        self._jobs = torch.from_numpy(jobs).to(self.dev)
        self.n_jobs = n

    def _weights_key(self):
        # writes through the arena (restore) bump flat's counter; in-place writes to a
        # Parameter (load_state_dict, `with torch.no_grad(): p.copy_(w)`) bump that
        # Parameter's own.  `p.data.copy_(w)` bumps neither (a `.data` alias carries a
        # fresh version counter): sync_weights() is the documented call after it
        return (self.arena.flat._version,) + tuple(op.conv.weight._version for op in self.trunk.convs)

    def sync_weights(self):
        """Re-pack the conv weights from the fp32 masters (one launch).  step() calls
        it itself when a version counter shows the masters were written from outside
        the step; after a write the counters cannot see -- through `p.data` or a raw
        pointer (ctypes, another library) -- the caller must call it before the next
        step() or eval forward."""
        self.trunk.pack_weights(force=True)
        self._packed_key = self._weights_key()

    def _sync_if_stale(self):
        if self.pack_in_adamw and self._weights_key() != self._packed_key:
            self.sync_weights()

    # ------------------------------------------------------------- DDP buckets
    def _buckets(self, bucket_mb, tail_mb=0.0):
        """Split the flat gradient into contiguous buckets; each closes after the
        backward of the conv whose weight is its last parameter.  The last bucket
        (stem / layer1, ready only when the backward ends: its all-reduce is not
        overlapped) is capped at tail_mb (tools/ddp_overlap.py models the tail)."""
        self.bucket_ends = []
        if not self._ddp:
            return
        sizes = [(off, p.numel()) for p, off in zip(self.arena.params, self.arena.offsets)]
        ends = plan_buckets(sizes, int(bucket_mb * 1e6 / 4), int(tail_mb * 1e6 / 4))
        ends[-1] = (ends[-1][0], self.arena.numel)   # the last bucket covers the alignment tail
        self.bucket_ends = [(self.arena.params[i], e) for i, e in ends]

    # ------------------------------------------------------------- the step
    def _forward_loss(self, rgb, depth_raw, bbox, K, gt_rot, gt_trans):
        st = stream()
        feat = self.trunk.forward(rgb, True, pack=False)
        raw = self.head.forward(feat, True, seed_dev=self.seed, salt=1)
        # F.normalize + pinhole + PoseLoss fwd/bwd + normalize bwd: one launch (the same
        # arithmetic as the rownorm_* / pinhole_depth / pose_loss_* entry points)
        call("geo_head_loss", raw, depth_raw, depth_raw.shape[1], depth_raw.shape[2], bbox, K,
             1 if K.dim() == 3 else 0, gt_rot, gt_trans, self.B, self.wr, self.wt, 0, self.rot, self.trans, self.loss,
             self.draw, self.dtrans, st)
        return raw

    def _head_backward(self):
        return self.head.backward(self.draw, self.arena.grad_of)

    def _optimizer(self):
        st = stream()
        if self._avg_pass:
            self.arena.grad.mul_(1.0 / self.world)   # post-all-reduce average (non power-of-two world)
        # (world > 1: the 1/world average of the all-reduced gradient is hp[6], applied
        # inside adamw_step; the norm partials see the sum, scaled there too)
        # step counter hp[5] += 1 and dropout seed += 1 ride on the norm-partials launch
        # (the seed is next read by the following step's forward)
        call("sumsq_partial_step", self.arena.grad, self.arena.numel, self.partials, NPART,
             self.hp[5:6], self.seed, st)
        if self.pack_in_adamw:   # + the packed conv weights the next step's forward reads
            call("adamw_step_packed", self.arena.flat, self.arena.grad, self.m, self.v, self.partials, NPART, self.hp,
                 self.norm, self.trunk.dt, self.trunk._desc_dev, self._jobs, self.n_jobs, st)
        else:
            call("adamw_step", self.arena.flat, self.arena.grad, self.m, self.v, self.arena.numel, self.partials,
                 NPART, self.hp, self.norm, st)

    def _pack(self):
        if not self.pack_in_adamw:
            self.trunk.pack_weights(force=True)

    def step_eager(self, data):
        """One training step without graphs (reference order of operations)."""
        self._sync_if_stale()
        if not self._ddp:
            return self.step_body(data, branch=True)
        self._pack()
        self._forward_loss(*data)
        dfeat = self._head_backward()
        self._backward_ddp(dfeat)
        self._optimizer()

    def step_body(self, data, branch=False):
        """The one-GPU step's launches, in order (what capture() records for world == 1;
        pose6d.steptime captures it for in-step kernel timing).  branch=True (the
        captured and eager one-GPU step) with POSE6D_HEAD_WGRAD_SIDE=1 (off by default:
        measured slower): the head's Linear weight gradients run on a side stream,
        overlapping the trunk backward, joined before the optimizer reads the
        gradients; otherwise the graph is one chain (pose6d.steptime splices its event
        nodes into a chain)."""
        self._pack()
        self._forward_loss(*data)
        side = self._side_stream() if branch and POSE6D_HEAD_WGRAD_SIDE else None
        dfeat = self.head.backward(self.draw, self.arena.grad_of, wgrad_stream=side)
        self.trunk.backward(dfeat, self.arena.grad_of)
        if side is not None:
            torch.cuda.current_stream().wait_stream(side)
        self._optimizer()

    def _side_stream(self):
        if not hasattr(self, "_side"):
            self._side = torch.cuda.Stream(device=self.dev)
        return self._side

    # ------------------------------------------------------------- DDP backward
    def _backward_ddp(self, dfeat):
        """Trunk backward with bucketed all-reduce: when the conv that completes a
        bucket is done, the bucket's all-reduce is enqueued on the comm stream
        (ordered after that point by an event) and overlaps the rest of backward."""
        red = BucketReducer(self.arena.grad, self.bucket_ends, self.pg, self._comm_stream())

        def on_conv(op):
            # gradients complete in arena order: after this conv, everything up to its
            # last parameter (weight, or bias if it has one) is final
            last = op.conv.bias if op.conv.bias is not None else op.conv.weight
            red.ready(self.arena.end_offset(last))

        self.trunk.backward(dfeat, self.arena.grad_of, on_conv_done=on_conv)
        red.finish()

    def _comm_stream(self):
        if not hasattr(self, "_comm"):
            self._comm = torch.cuda.Stream(device=self.dev)
        return self._comm

    # ------------------------------------------------------------- graphs
    def capture(self, data, warmup=2):
        """Capture the step.  world == 1: one graph.  world > 1: the forward +
        backward as graph segments cut where a gradient bucket completes, and the
        optimizer as a graph of its own (the all-reduces run between replays)."""
        self._sync_if_stale()
        s = torch.cuda.Stream(device=self.dev)
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(warmup):
                self.step_eager(data)
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        if not self._ddp:
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, capture_error_mode="thread_local"):
                self.step_body(data, branch=True)
            self.graphs = [g]
        else:
            self.graphs = self._capture_segments(data)
        torch.cuda.synchronize()

    def _capture_segments(self, data):
        """[(graph, buckets it completes)] for forward + backward, then the optimizer
        graph.  Segment boundaries are the launches after which on_conv_done makes
        a bucket ready: exactly where the eager path issues that bucket."""
        pool = torch.cuda.graph_pool_handle()
        ends = [e for _, e in self.bucket_ends]
        segs = []
        st = {"g": None, "next": 0}
        cs = torch.cuda.Stream(device=self.dev)
        cs.wait_stream(torch.cuda.current_stream())

        # thread-local capture: the RCCL watchdog thread keeps querying the events of
        # earlier all-reduces while these segments are captured; under the default
        # (global) mode such a call from another thread is illegal during a capture and
        # the watchdog aborts the process
        def begin():
            st["g"] = torch.cuda.CUDAGraph()
            st["g"].capture_begin(pool=pool, capture_error_mode="thread_local")

        def cut(upto):
            # the last bucket (ending at the arena end) always goes out after the
            # final segment, which therefore never comes out empty
            first = st["next"]
            while st["next"] < len(ends) - 1 and ends[st["next"]] <= upto:
                st["next"] += 1
            if st["next"] > first:
                st["g"].capture_end()
                segs.append((st["g"], (first, st["next"])))
                begin()

        def on_conv(op):
            last = op.conv.bias if op.conv.bias is not None else op.conv.weight
            cut(self.arena.end_offset(last))

        with torch.cuda.stream(cs):
            begin()
            self._pack()
            self._forward_loss(*data)
            dfeat = self._head_backward()
            self.trunk.backward(dfeat, self.arena.grad_of, on_conv_done=on_conv)
            st["g"].capture_end()
            segs.append((st["g"], (st["next"], len(ends))))
            opt = torch.cuda.CUDAGraph()
            opt.capture_begin(pool=pool, capture_error_mode="thread_local")
            self._optimizer()
            opt.capture_end()
        torch.cuda.current_stream().wait_stream(cs)
        self._red = BucketReducer(self.arena.grad, self.bucket_ends, self.pg, self._comm_stream())
        return segs + [(opt, None)]

    def step(self, data=None):
        self._sync_if_stale()
        if self.graphs is None:
            return self.step_eager(data)
        if not self._ddp:
            self.graphs[0].replay()
            return
        red = self._red
        red.reset()
        ends = red.ends
        for g, buckets in self.graphs[:-1]:
            g.replay()
            lo, hi = buckets
            if hi > lo:
                red.ready(ends[hi - 1])
        red.finish()
        self.graphs[-1][0].replay()

    def snapshot(self):
        """Device copies of everything a step changes (parameters, AdamW moments and
        step, dropout seed, BN buffers) -- restore() rewinds to it in place, so a
        captured graph keeps running on the same storage."""
        bufs = [b for n, b in self.model.named_buffers() if "running" in n or "num_batches" in n]
        return [t.clone() for t in (self.arena.flat, self.m, self.v, self.hp, self.seed, *bufs)]

    def restore(self, snap):
        bufs = [b for n, b in self.model.named_buffers() if "running" in n or "num_batches" in n]
        with torch.no_grad():
            for dst, src in zip((self.arena.flat, self.m, self.v, self.hp, self.seed, *bufs), snap):
                dst.copy_(src)

    def set_lr(self, lr):
        self.hp[0].fill_(lr)

    # ------------------------------------------------------------- checkpoints
    def _torch_adamw(self):
        lr, b1, b2, eps, wd = (float(v) for v in self.hp[:5].tolist())
        return torch.optim.AdamW(self.model.parameters(), lr=lr, betas=(b1, b2), eps=eps, weight_decay=wd)

    def optimizer_state_dict(self):
        """The AdamW state as torch.optim.AdamW(model.parameters()).state_dict()
        lays it out -- the `optimizer_state_dict` entry the reference's training
        script saves and resumes from (train_rgbd_geometric.py:65,82,154)."""
        opt = self._torch_adamw()
        step = float(self.hp[5].item())
        if step > 0:
            for p in self.model.parameters():
                o, n = self.arena.offsets[self.arena._index_of(p)], p.numel()
                opt.state[p] = {"step": torch.tensor(step), "exp_avg": self.m[o:o + n].view_as(p).clone(),
                                "exp_avg_sq": self.v[o:o + n].view_as(p).clone()}
        return opt.state_dict()

    def load_optimizer_state_dict(self, sd):
        """Inverse of optimizer_state_dict(): accepts a torch AdamW state_dict over
        model.parameters() (e.g. a reference checkpoint's optimizer_state_dict)."""
        opt = self._torch_adamw()
        opt.load_state_dict(sd)
        g = opt.param_groups[0]
        self.hp[:5].copy_(torch.tensor([g["lr"], g["betas"][0], g["betas"][1], g["eps"], g["weight_decay"]]))
        step = 0.0
        with torch.no_grad():
            self.m.zero_()
            self.v.zero_()
            for p in self.model.parameters():
                st = opt.state.get(p)
                if not st:
                    continue
                o, n = self.arena.offsets[self.arena._index_of(p)], p.numel()
                self.m[o:o + n].copy_(st["exp_avg"].reshape(-1))
                self.v[o:o + n].copy_(st["exp_avg_sq"].reshape(-1))
                step = float(st["step"])
        self.hp[5].fill_(step)

    def checkpoint(self, epoch, best_acc=0.0, curr_acc=0.0, **extra):
        """The reference's checkpoint dict (train_rgbd_geometric.py:151-157): model
        state_dict with the reference's keys (OIHW fp32 masters), torch-AdamW
        optimizer state, epoch, best / current accuracy (+ e.g. curr_add)."""
        return {"epoch": epoch, "model_state_dict": self.model.state_dict(),
                "optimizer_state_dict": self.optimizer_state_dict(), "best_acc": best_acc, "curr_acc": curr_acc,
                **extra}

    def load_checkpoint(self, ckpt):
        """Resume from a reference-format checkpoint (train_rgbd_geometric.py:79-84):
        parameters / BN buffers are copied into the flat arena in place, so the
        captured graph keeps running on them.  Returns the next epoch."""
        self.model.load_state_dict(ckpt["model_state_dict"])
        if "optimizer_state_dict" in ckpt:
            self.load_optimizer_state_dict(ckpt["optimizer_state_dict"])
        return ckpt.get("epoch", -1) + 1
