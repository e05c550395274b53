"""Data-parallel paths with world_size 2 over gloo on the CPU:
the bucketed gradient all-reduce of training and the sharded ADD evaluation.
The GPU-side producers (kernels) are stood in for by plain tensors / the oracle;
what is tested is the host logic that runs unchanged over RCCL on MI355X."""
import os
import tempfile

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

WORLD = 2


def _run(fn, *args):
    d = tempfile.mkdtemp()
    init = "file://" + os.path.join(d, "rdv")
    out = os.path.join(d, "out")
    mp.spawn(_entry, args=(fn, init, out, args), nprocs=WORLD, join=True)
    return [torch.load(f"{out}.{r}", weights_only=True) for r in range(WORLD)]


def _entry(rank, fn, init, out, args):
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    dist.init_process_group("gloo", init_method=init, rank=rank, world_size=WORLD)
    try:
        torch.save(fn(rank, *args), f"{out}.{rank}")
    finally:
        dist.destroy_process_group()


def test_plan_buckets_covers_arena():
    from pose6d.dist import plan_buckets
    rng = np.random.default_rng(0)
    sizes, off = [], 0
    for _ in range(200):
        n = int(rng.integers(1, 300_000))
        sizes.append((off, n))
        off += (n + 63) // 64 * 64
    ends = plan_buckets(sizes, 1_000_000)
    e = [x for _, x in ends]
    assert e == sorted(e) and len(set(e)) == len(e)
    assert e[-1] == sizes[-1][0] + sizes[-1][1]
    starts = [0] + e[:-1]
    assert all(b - a >= 1_000_000 for a, b in zip(starts[:-1], e[:-1]))   # only the last may be short
    for i, x in ends:
        assert x == sizes[i][0] + sizes[i][1]                            # buckets close at tensor ends


@pytest.mark.parametrize("tail", [50_000, 300_000, 900_000])
def test_plan_buckets_tail_cap(tail):
    """tail_elems: the last bucket is split at a tensor end so that it holds at most
    `tail` elements (or only the last tensor); the other buckets are unchanged."""
    from pose6d.dist import plan_buckets
    rng = np.random.default_rng(1)
    sizes, off = [], 0
    for _ in range(120):
        n = int(rng.integers(1, 200_000))
        sizes.append((off, n))
        off += n
    base = plan_buckets(sizes, 2_500_000)
    ends = plan_buckets(sizes, 2_500_000, tail)
    e = [x for _, x in ends]
    assert e == sorted(e) and len(set(e)) == len(e) and e[-1] == off
    for i, x in ends:
        assert x == sizes[i][0] + sizes[i][1]
    lo = base[-2][1] if len(base) > 1 else 0
    if off - lo > tail:
        assert ends[:-2] == base[:-1] and len(ends) == len(base) + 1
        assert off - e[-2] <= tail or e[-2] == sizes[-2][0] + sizes[-2][1]
        # the shortest suffix within the cap: one tensor more would exceed it
        k = [i for i, _ in ends][-2]
        assert off - (sizes[k][0]) > tail or k == [i for i, _ in base][-2] + 1
    else:
        assert ends == base


def _reducer_worker(rank, n, ends):
    from pose6d.dist import BucketReducer
    g = torch.arange(n, dtype=torch.float32) * (rank + 1)
    red = BucketReducer(g, [(None, e) for e in ends], group=None)
    issued_after = []
    for upto in (0, ends[0] - 1, ends[0], ends[1] + 5):   # backward finishing prefixes
        red.ready(upto)
        issued_after.append(len(red.issued))
    red.finish()
    return {"grad": g, "issued_after": torch.tensor(issued_after), "issued": torch.tensor(red.issued)}


def test_bucket_reducer_gloo_world2():
    n, ends = 1000, [300, 620, 1000]
    res = _run(_reducer_worker, n, ends)
    expect = torch.arange(n, dtype=torch.float32) * 3     # rank 0 (x1) + rank 1 (x2)
    for r in res:
        assert torch.equal(r["grad"], expect)
        assert r["issued_after"].tolist() == [0, 0, 1, 2]     # a bucket goes out exactly when its prefix is done
        assert r["issued"].tolist() == [[0, 300], [300, 620], [620, 1000]]


def _add_worker(rank, B):
    from models.add_loss import ADDLoss
    from oracle import add_loss as OA
    from pose6d.dist import gather_samples, shard
    from tests.synth import LINEMOD_OBJ_IDS, make_poses, synthetic_meshes
    pts, diam = synthetic_meshes(300, seed=5)
    rng = np.random.default_rng(9)
    ids = np.array([LINEMOD_OBJ_IDS[i % 13] for i in range(B)], np.int64)
    if B > 3:
        ids[3] = 99                                        # an unknown object is skipped
    pr, pt, gr, gt = make_poses(rng, B)
    lo, hi = shard(B, rank, WORLD)
    # stand-in for pose6d_add_eval on this rank's shard (the oracle computes the same values)
    s = OA.per_sample(pts, diam, pr[lo:hi], pt[lo:hi], gr[lo:hi], gt[lo:hi], ids[lo:hi])
    valid = torch.tensor(s["valid"], dtype=torch.int32)
    add = torch.zeros(hi - lo, dtype=torch.float64)
    adds = torch.zeros(hi - lo, dtype=torch.float64)
    corr = torch.zeros(hi - lo, dtype=torch.int32)
    vi = torch.nonzero(valid).flatten()
    add[vi] = torch.tensor(s["add"], dtype=torch.float64)
    adds[vi] = torch.tensor(s["adds"], dtype=torch.float64)
    corr[vi] = torch.tensor(s["correct"], dtype=torch.int32)
    full = gather_samples([add, adds, valid, corr])
    got = ADDLoss.aggregate(*full)
    ref = OA.eval_metrics(pts, diam, pr, pt, gr, gt, ids)
    return {"got": torch.tensor([got["add_mean"], got["add_s_mean"], got["add_01d_acc"]], dtype=torch.float64),
            "ref": torch.tensor([ref["add_mean"], ref["add_s_mean"], ref["add_01d_acc"]], dtype=torch.float64),
            "n": torch.tensor(full[0].shape[0])}


@pytest.mark.parametrize("B", [7, 1])
def test_sharded_add_eval_gloo_world2(B):
    """Uneven (7 = 4 + 3) and empty-shard (1 = 1 + 0) splits: every rank ends with
    the eval_metrics of the whole batch."""
    for r in _run(_add_worker, B):
        assert int(r["n"]) == B
        np.testing.assert_allclose(r["got"].numpy(), r["ref"].numpy(), rtol=1e-12)
