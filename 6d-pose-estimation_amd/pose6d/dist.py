"""Data-parallel plumbing of the hot path, one process per GPU.

* BucketReducer: the gradient all-reduce of training.  The flat fp32 gradient
  arena is cut into contiguous buckets (~25 MB, in gradient-completion order);
  as backward finishes each prefix, the buckets inside it are all-reduced
  (SUM) on a communication stream ordered after the producing stream by an
  event, overlapping the rest of backward.  RCCL over xGMI on the GPU box
  (backend 'nccl'), gloo in the CPU tests.
* shard / gather_samples: the ADD / ADD-S evaluation shards independent samples
  over ranks and all-gathers the per-sample results, so rank 0 aggregates in
  the reference's order (mean over samples, add_loss.py:197-201).
"""
import torch
import torch.distributed as dist


def plan_buckets(sizes, bucket_elems, tail_elems=0):
    """Bucket end offsets over a flat buffer holding tensors of `sizes` elements
    (with the given per-tensor offsets folded in by the caller): a bucket closes
    at the first tensor end that makes it >= bucket_elems; the last bucket ends
    at the buffer end.  tail_elems > 0: a last bucket larger than that is split at
    the tensor end that leaves the longest suffix of at most tail_elems (or the last
    tensor alone) -- the last bucket is only ready when the backward ends, so its
    all-reduce is the step's unhidden tail.  Returns [(tensor_index, end_offset)]."""
    ends, start, off = [], 0, 0
    for i, (o, n) in enumerate(sizes):
        end = o + n
        if end - start >= bucket_elems:
            ends.append((i, end))
            start = end
        off = end
    if sizes and (not ends or ends[-1][1] != off):
        ends.append((len(sizes) - 1, off))
    if tail_elems > 0 and ends:
        first = ends[-2][0] + 1 if len(ends) > 1 else 0   # the last bucket's first tensor
        lo = ends[-2][1] if len(ends) > 1 else 0
        if off - lo > tail_elems:
            cut = None
            for i in range(first, len(sizes) - 1):
                e = sizes[i][0] + sizes[i][1]
                if off - e <= tail_elems:
                    cut = (i, e)
                    break
            if cut is None and len(sizes) - 1 > first:
                i = len(sizes) - 2
                cut = (i, sizes[i][0] + sizes[i][1])
            if cut is not None:
                ends.insert(len(ends) - 1, cut)
    return ends


class BucketReducer:
    """Issues SUM all-reduces of grad[start:end] per bucket as soon as the
    completed prefix of the flat gradient covers the bucket (ready(upto)),
    then finish() issues the rest and waits.  The caller divides by the world
    size (folded into the optimizer step)."""

    def __init__(self, grad, bucket_ends, group=None, comm_stream=None):
        self.grad = grad
        self.ends = [e for _, e in bucket_ends]
        self.group = group
        self.comm = comm_stream
        self.reset()

    def reset(self):
        self.next = 0
        self.start = 0
        self.handles = []
        self.issued = []

    def ready(self, upto):
        """Every gradient element below `upto` is final on the current stream."""
        while self.next < len(self.ends) and self.ends[self.next] <= upto:
            end = self.ends[self.next]
            view = self.grad[self.start:end]
            if self.comm is not None:
                ev = torch.cuda.Event()
                ev.record(torch.cuda.current_stream())
                with torch.cuda.stream(self.comm):
                    self.comm.wait_event(ev)
                    self.handles.append(dist.all_reduce(view, group=self.group, async_op=True))
            else:
                self.handles.append(dist.all_reduce(view, group=self.group, async_op=True))
            self.issued.append((self.start, end))
            self.start = end
            self.next += 1

    def finish(self):
        self.ready(self.grad.numel())
        for h in self.handles:
            h.wait()
        if self.comm is not None:
            torch.cuda.current_stream().wait_stream(self.comm)
        self.handles = []


def shard(n, rank, world):
    """Contiguous [lo, hi) sample range of `rank` (sizes differ by at most one)."""
    q, r = divmod(n, world)
    lo = rank * q + min(rank, r)
    return lo, lo + q + (1 if rank < r else 0)


def gather_samples(tensors, group=None):
    """All-gather per-sample tensors (first dim = this rank's sample count, which
    may differ between ranks) into full-length tensors on every rank, in rank
    order (= sample order when the batch was split with `shard`)."""
    world = dist.get_world_size(group)
    dev = tensors[0].device
    n = torch.tensor([tensors[0].shape[0]], dtype=torch.int64, device=dev)
    counts = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(counts, n, group=group)
    counts = [int(c.item()) for c in counts]
    width = max(max(counts), 1)
    out = []
    for t in tensors:
        pad = torch.zeros((width,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
        pad[:t.shape[0]] = t
        parts = [torch.empty_like(pad) for _ in range(world)]
        dist.all_gather(parts, pad, group=group)
        out.append(torch.cat([p[:c] for p, c in zip(parts, counts)]))
    return out
