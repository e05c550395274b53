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
