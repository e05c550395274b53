"""CPU-side checks of the C ABI boundary: the library loads, exports every
symbol include/pose6d.h declares, and the product refuses CPU tensors."""
import ctypes
import os

import pytest
import torch

from pose6d import _lib


def test_library_exports_every_header_symbol():
    lib = _lib.load()
    names = _lib.symbols()
    assert len(names) >= 10
    for n in names:
        assert hasattr(lib, n), n
    assert lib.pose6d_version() >= 1
    assert isinstance(lib.pose6d_last_error(), bytes)


def test_header_has_no_torch_types():
    import re
    src = re.sub(r"/\*.*?\*/", "", open(_lib.HEADER).read(), flags=re.S)
    for bad in ("torch", "at::", "Tensor", "c10"):
        assert bad not in src


def test_no_cpu_fallback():
    from models.pose_loss import PoseLoss
    with pytest.raises(_lib.Pose6dError):
        PoseLoss()(torch.randn(2, 4), torch.randn(2, 3), torch.randn(2, 4), torch.randn(2, 3))


def test_invalid_args_reported_without_gpu():
    lib = _lib.load()
    rc = lib.pose6d_rownorm_fwd(None, None, 4, 0, 0, None)   # D = 0 -> EINVAL before any launch
    assert rc == 1
    assert b"bad D" in lib.pose6d_last_error()


def test_conv_plan_query_reports_split_k():
    """pose6d_conv_variant (host-only plan query): (splits << 16) | (stages << 12) |
    (fast << 8) | (mode << 4) | tile.  Split-K is taken by default only for long-K convs
    on grids of <= 256 64x64 tiles (layer4 at batch 32); data gradients never split by
    default (fused and separate backward stay one plan, and the backward entry points take
    no split-K workspace); pose6d_conv_splitk_workspace sizes the caller's scratch."""
    from pose6d._lib import DT_BF16, DT_F32, query

    def splits(dt, pas, N, H, Cin, Cout, k, s):
        p = k // 2
        Ho = (H + 2 * p - k) // s + 1
        return query("conv_variant", dt, pas, N, H, H, Cin, Cout, k, k, s, p, Ho, Ho) >> 16

    for dt in (DT_BF16, DT_F32):
        assert splits(dt, 0, 32, 7, 512, 512, 3, 1) == 2      # layer4 3x3: 72 K-steps, 200 tiles
        assert splits(dt, 0, 32, 7, 2048, 512, 1, 1) == 2     # layer4 2048 -> 512 1x1
        assert splits(dt, 0, 32, 56, 64, 256, 1, 1) == 1      # layer1: big grid
        assert splits(dt, 0, 32, 14, 256, 1024, 1, 1) == 1    # short K
    for dt in (DT_BF16, DT_F32):                             # data gradients: split only when tuned
        assert splits(dt, 1, 32, 7, 512, 512, 3, 1) == 1
    # small grids (batch 1-2, <= 64 64x64 tiles) with >= 16 K-steps: four splits (round 6)
    for dt in (DT_BF16, DT_F32):
        assert splits(dt, 0, 1, 7, 512, 512, 3, 1) == 4       # layer4 3x3 at B = 1: 8 tiles
        assert splits(dt, 0, 1, 14, 1024, 256, 1, 1) == 4     # 16 K-steps (bf16), 16 tiles
        assert splits(dt, 0, 1, 7, 512, 2048, 1, 1) == (1 if dt == DT_BF16 else 4)   # 8 (bf16) / 16 (fp32) K-steps
        assert splits(dt, 0, 2, 14, 256, 256, 3, 1) == 4      # B = 2: 32 tiles
        assert splits(dt, 0, 32, 7, 512, 512, 3, 1) == 2      # batch 32 unchanged

    # the split-K workspace a plan needs (caller-provided: 32 KiB of counters + partial tiles)
    def ws(dt, pas, N, H, Cin, Cout, k, s):
        p = k // 2
        Ho = (H + 2 * p - k) // s + 1
        return query("conv_splitk_workspace", dt, pas, N, H, H, Cin, Cout, k, k, s, p, Ho, Ho)
    assert ws(DT_BF16, 0, 32, 7, 512, 512, 3, 1) == 32768 + 200 * 2 * 64 * 64 * 4
    assert ws(DT_BF16, 0, 32, 56, 64, 256, 1, 1) == 0
    assert ws(DT_F32, 1, 32, 7, 512, 512, 3, 1) == 0


def test_dual_eval_launch_rejects_split_k_geometry():
    """pose6d_conv2d_fwd_act_dual refuses a pair whose separate launches would split K
    (bit identity with them needs unsplit K loops), before touching any pointer."""
    lib = _lib.load()
    # fp32 layer4 downsampling block at batch 4: the 1024 -> 2048 downsample splits K
    rc = lib.pose6d_conv2d_fwd_act_dual(_lib.DT_F32, None, None, None, None, None, 4, 7, 7, 512, 2048, 14, 14, 1024,
                                        2, ctypes.c_void_p(1), ctypes.c_void_p(1), ctypes.c_void_p(1),
                                        ctypes.c_void_p(1), 1, None)
    assert rc == 1
    assert b"split K" in lib.pose6d_last_error()


def test_add_eval_table_arguments_checked_without_gpu():
    """pose6d_add_neighbors / pose6d_add_eval_nbr refuse a neighbour count other than 8 / 16 / 32,
    meshes beyond the uint16 index range and a misaligned table, before any launch."""
    lib = _lib.load()
    one = ctypes.c_void_p(16)
    rc = lib.pose6d_add_neighbors(one, one, one, 1, 100, 12, one, None)
    assert rc == 1 and b"K must be 8, 16 or 32" in lib.pose6d_last_error()
    rc = lib.pose6d_add_neighbors(one, one, one, 1, 70000, 16, one, None)
    assert rc == 1 and b"bad table sizes" in lib.pose6d_last_error()
    args = [one] * 5 + [1] + [one] * 5 + [1, 100]
    rc = lib.pose6d_add_eval_nbr(*args, ctypes.c_void_p(24), 16, *([one] * 7), None)   # 8-byte aligned table
    assert rc == 1 and b"16-byte alignment" in lib.pose6d_last_error()
    rc = lib.pose6d_add_eval_nbr(*args, one, 24, *([one] * 7), None)
    assert rc == 1 and b"K in {8, 16, 32}" in lib.pose6d_last_error()
