"""Shared plumbing of the drop-in PoseNet modules: engine bookkeeping, compute
dtype, and the device-side dropout seed."""
import os

import torch
import torch.nn as nn

from . import autograd
from .head import HeadEngine
from .trunk import TrunkEngine

_DTYPE_ENV = {"fp32": torch.float32, "f32": torch.float32, "float32": torch.float32, "bf16": torch.bfloat16,
              "bfloat16": torch.bfloat16}


def default_compute_dtype():
    return _DTYPE_ENV[os.environ.get("POSE6D_COMPUTE_DTYPE", "fp32").lower()]


class EngineModel(nn.Module):
    """nn.Module whose children hold the reference's parameters while the math
    runs in pose6d engines (not submodules: state_dict keys stay the reference's)."""

    def _p6_init(self):
        self._p6_dtype = default_compute_dtype()
        self._p6_engines = {}
        self.register_buffer("_p6_seed", torch.tensor([torch.initial_seed() & 0x7FFFFFFFFFFF], dtype=torch.int64),
                             persistent=False)

    def set_compute_dtype(self, dtype):
        """torch.float32 (reference numerics) or torch.bfloat16 (trunk activations
        and MFMA operands in bf16, fp32 accumulation / BN statistics / heads)."""
        self._p6_dtype = dtype
        return self

    @property
    def compute_dtype(self):
        return self._p6_dtype

    def _engine(self, name, factory):
        eng = self._p6_engines.get(name)
        if eng is None:
            eng = factory()
            self._p6_engines[name] = eng
        return eng

    def _run_trunk(self, name, seq, x, in_channels, kind="resnet50"):
        eng = self._engine(name, lambda: TrunkEngine(seq, in_channels, kind))
        eng.set_dtype(self._p6_dtype)
        # trunk features only ever feed the model's own heads / fusion: no copy
        return autograd.run(eng, x, self.training, list(seq.parameters()), copy=False)

    def _run_head(self, name, seq, x, salt, copy=True):
        """copy=False: the output is consumed right away by another op (normalize,
        pinhole) and never reaches the caller, so no-grad forwards skip the copy."""
        eng = self._engine(name, lambda: HeadEngine(seq))
        return autograd.run(eng, x, self.training, list(seq.parameters()), copy=copy, seed_dev=self._p6_seed,
                            salt=salt)

    def _advance_seed(self):
        if self.training:
            with torch.no_grad():
                self._p6_seed.add_(1)

    def engines(self):
        return dict(self._p6_engines)

    def sync_weights(self):
        """Re-pack every trunk engine's compute-dtype conv weights from the fp32
        masters now.  Forwards re-pack by themselves after writes torch's version
        counters record (load_state_dict, optimizer steps, in-place ops on a
        Parameter); a write through `p.data` (a `.data` alias has a version counter
        of its own) or a raw pointer is invisible to them and needs this call."""
        for eng in self._p6_engines.values():
            if isinstance(eng, TrunkEngine) and getattr(eng, "_shape", None) is not None:
                eng.pack_weights(force=True)
        return self
