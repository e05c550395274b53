"""pose6d — MI355X-native runtime for the SFR-Vision/6d-pose-estimation hot path.

Layers:
  _lib      ctypes binding of libpose6d.so (C ABI in include/pose6d.h)
  ops       torch.autograd.Functions over the C ABI (no CPU fallback)
  trunk     ResNet50 trunk engine: NHWC activations, packed weights, fused BN
  train     whole-step trainer (fwd + loss + bwd + clip + AdamW), hipGraph-captured
  ddp       batch-sharded data parallel over RCCL
The drop-in reference API lives in ../models (same module/class names).
"""
from ._lib import Pose6dError, load  # noqa: F401
