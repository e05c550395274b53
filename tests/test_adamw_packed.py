"""AdamW that emits the packed conv weights (pose6d_adamw_step_packed): the trainer's
optimizer launch writes each conv's compute-dtype copies (wp / wt) from the updated
fp32 masters, so the step has no packing launch.  Checked here:
  * (CPU) the host-built job table covers every parameter exactly once -- plain
    ranges between the convs, tiles of 64 filters x a channel group (every tap) over
    each conv's [O][I*KH*KW] master;
  * (GPU) bit-identity with the previous layout (pack_weights at the start of every
    step + plain adamw_step): masters, moments and every packed copy equal after
    graph-replayed steps, across a restore() and a load_state_dict() from outside
    the step (both must trigger a re-pack)."""
import copy
import warnings

import numpy as np
import pytest
import torch

from pose6d._lib import query
from pose6d.trunk import _DESC


def _jobs(descs, base, n):
    args = (descs.ctypes.data, len(descs), base, n)
    cnt = query("adamw_packed_jobs", *args, None, 0)
    assert cnt > 0
    jobs = np.zeros((cnt, 4), dtype=np.int32)
    assert query("adamw_packed_jobs", *args, jobs.ctypes.data, cnt) == cnt
    return jobs


def test_packed_jobs_cover_every_parameter_once():
    # (O, I, k) of a few conv shapes incl. the stem's odd reduction length (3 * 49)
    shapes = [(64, 3, 7), (64, 64, 1), (64, 64, 3), (256, 64, 1), (128, 256, 1), (512, 1024, 1), (48, 20, 3)]
    base = 1 << 20   # a fake device address: the builder only compares pointers
    rec = np.zeros(len(shapes), dtype=_DESC)
    off = 100   # a plain range before the first conv
    offs = []
    for i, (O, I, k) in enumerate(shapes):
        off = (off + 63) // 64 * 64
        ip = (I + 7) // 8 * 8
        rec[i] = (base + 4 * off, 0x1000, 0, O, I, ip, k, k, (k * k * ip + 31) // 32 * 32, k, 0, 0)
        offs.append((off, O * I * k * k))
        off += O * I * k * k + 37   # + a gap of plain parameters
    n = (off + 63) // 64 * 64
    order = np.random.default_rng(0).permutation(len(shapes))   # the builder sorts by address
    jobs = _jobs(rec[order].copy(), base, n)
    seen = np.zeros(n, dtype=np.int32)
    for kind, a, b, c in jobs:
        if kind == 0:
            assert 0 < b - a <= 4096
            seen[a:b] += 1
        else:
            assert kind == 1
            O, I, k = shapes[order[a]]
            R, o0, taps = I * k * k, offs[order[a]][0], k * k
            cw = 64 if taps == 1 else max(1, min(8, 128 // taps))   # optim.hip tile_channels
            assert b % 64 == 0 and c % cw == 0 and b < O and c < I
            for o in range(b, min(b + 64, O)):
                seen[o0 + o * R + c * taps:o0 + o * R + min(c + cw, I) * taps] += 1
    assert (seen == 1).all(), np.flatnonzero(seen != 1)[:10]


def test_packed_jobs_reject_bad_tables():
    rec = np.zeros(2, dtype=_DESC)
    base = 1 << 20
    rec[0] = (base, 0x1000, 0, 64, 64, 64, 1, 1, 64, 1, 0, 0)
    rec[1] = (base + 4 * 64, 0x1000, 0, 64, 64, 64, 1, 1, 64, 1, 0, 0)   # overlaps conv 0
    assert query("adamw_packed_jobs", rec.ctypes.data, 2, base, 1 << 16, None, 0) < 0
    rec[1] = (base + 4 * 4098, 0x1000, 0, 64, 64, 64, 1, 1, 64, 1, 0, 0)
    assert query("adamw_packed_jobs", rec.ctypes.data, 2, base, 8192, None, 0) < 0   # past the end
    rec[1] = (base + 4 * 4097, 0x1000, 0, 64, 64, 64, 1, 1, 64, 1, 0, 0)
    assert query("adamw_packed_jobs", rec.ctypes.data, 2, base, 1 << 16, None, 0) < 0   # misaligned
    # a filter whose taps exceed the kernel's 128-column LDS tile (13 x 13 = 169) is refused
    one = np.zeros(1, _DESC)
    one[0] = (base, 0x1000, 0, 8, 8, 8, 13, 13, 13 * 13 * 8, 13, 0, 0)
    assert query("adamw_packed_jobs", one.ctypes.data, 1, base, 1 << 16, None, 0) < 0
    one[0] = (base, 0x1000, 0, 8, 8, 8, 11, 11, 11 * 11 * 8, 11, 0, 0)   # 121 taps fit
    assert query("adamw_packed_jobs", one.ctypes.data, 1, base, 1 << 16, None, 0) > 0


def _pair(dtype, B=4):
    from models.pose_net_rgbd_geometric import PoseNetRGBDGeometric
    from pose6d.train import RGBDGeometricTrainer
    warnings.simplefilter("ignore")
    torch.manual_seed(0)
    m0 = PoseNetRGBDGeometric(pretrained=False)
    out = []
    for packed in (True, False):
        m = copy.deepcopy(m0).cuda()
        out.append(RGBDGeometricTrainer(m, B, dtype=dtype, pack_in_adamw=packed))
    return out


def _assert_same(a, b, what):
    """a: packed by its AdamW launch; b: the packing-pass layout, whose copies hold the
    PREVIOUS masters until its next step packs them -- packed here from its masters."""
    assert torch.equal(a.arena.flat, b.arena.flat), f"{what}: masters differ"
    assert torch.equal(a.m, b.m) and torch.equal(a.v, b.v), f"{what}: moments differ"
    b.trunk.pack_weights(force=True)
    torch.cuda.synchronize()
    for i, (x, y) in enumerate(zip(a.trunk.convs, b.trunk.convs)):
        assert torch.equal(x.wp, y.wp), f"{what}: conv {i} wp differs"
        if x.wt is not None:
            assert torch.equal(x.wt, y.wt), f"{what}: conv {i} wt differs"


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_packed_adamw_bit_identical_to_pack_pass(dtype):
    from bench import synth_batch
    trs = _pair(dtype)
    data = synth_batch(4, torch.device("cuda"), seed=11)
    snaps = [t.snapshot() for t in trs]
    for t, s in zip(trs, snaps):
        t.capture(data, warmup=1)
        t.restore(s)          # a write through the arena: re-packed before the next step
    for step in range(3):
        for t in trs:
            t.step()
        torch.cuda.synchronize()
        _assert_same(trs[0], trs[1], f"step {step}")
    # a write through the Parameters (load_state_dict of other weights)
    torch.manual_seed(1)
    from models.pose_net_rgbd_geometric import PoseNetRGBDGeometric
    sd = PoseNetRGBDGeometric(pretrained=False).state_dict()
    for t in trs:
        t.model.load_state_dict(sd)
        t.step()
    torch.cuda.synchronize()
    _assert_same(trs[0], trs[1], "after load_state_dict")
    # an in-place write to a Parameter under no_grad bumps its version counter: seen
    torch.manual_seed(2)
    w = torch.randn_like(trs[0].trunk.convs[5].conv.weight)
    for t in trs:
        with torch.no_grad():
            t.trunk.convs[5].conv.weight.copy_(w)
        t.step()
    torch.cuda.synchronize()
    _assert_same(trs[0], trs[1], "after an in-place Parameter write")
    # a write through `.data` is invisible to the version counters (a `.data` alias has
    # its own): the documented contract is an explicit sync_weights() before the next step
    w = torch.randn_like(trs[0].trunk.convs[7].conv.weight)
    for t in trs:
        t.trunk.convs[7].conv.weight.data.copy_(w)
        t.sync_weights()
        t.step()
    torch.cuda.synchronize()
    _assert_same(trs[0], trs[1], "after p.data.copy_ + sync_weights()")
