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
