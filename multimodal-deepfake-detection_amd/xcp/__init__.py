"""xcp -- MI355X-native (gfx950 HIP) runtime for the Xception + LSTM clip path.

Layout:
  csrc/      hand-written HIP kernels + the C ABI (declared in include/xcp.h)
  build.py   hipcc build of the in-tree libxcp.so
  _lib.py    ctypes binding of the C ABI (fails loudly when the library is missing)
  ops.py        typed wrappers over torch device tensors
  torch_ops.py  torch.library custom ops (namespace xcp) with fake kernels + autograd
  modules.py    nn.Conv2d / BatchNorm2d / MaxPool2d subclasses running those ops
  engine.py     whole-backbone fused forward/backward executor + autograd node
  lstm.py       nn.LSTM drop-in on the fused LSTM kernels
  ddp.py        one-process-per-GPU data parallelism over RCCL
  optim.py      fused clip_grad_norm_ + Adam (a torch.optim.Optimizer)
  heads.py      ArcFace head / CB-focal loss on HIP kernels; metrics.py: ROC / EER / pAUC

Precision of the backbone (activations / GEMM operands; accumulation is fp32, master
weights fp32, BN statistics fp64):
  * ``set_compute_dtype("bf16"|"fp32")`` / ``XCP_DTYPE=bf16|fp32``: that dtype;
  * otherwise fp32 (the reference's precision, train_audio.py), except inside an active
    ``torch.autocast("cuda")`` region (train_visual.py:567 / train_au_face.py:664), where the
    backbone computes in bf16 -- the kernels' reduced precision (autocast's own fp16 has no
    gfx950 kernel here; bf16 needs no loss scaling, a GradScaler stays harmless).
"""
import os
from contextlib import contextmanager

import torch

_DTYPES = {"bf16": torch.bfloat16, "bfloat16": torch.bfloat16, "fp32": torch.float32, "float32": torch.float32}
_env = os.environ.get("XCP_DTYPE", "").lower()
_compute_dtype = _DTYPES[_env] if _env else None


def compute_dtype():
    if _compute_dtype is not None:
        return _compute_dtype
    return torch.bfloat16 if torch.is_autocast_enabled("cuda") else torch.float32


def set_compute_dtype(dt):
    """Fix the backbone's compute dtype (None: back to the default rule above)."""
    global _compute_dtype
    if isinstance(dt, str):
        dt = _DTYPES[dt.lower()]
    if dt not in (torch.float32, torch.bfloat16, None):
        raise ValueError("compute dtype must be torch.float32 or torch.bfloat16")
    _compute_dtype = dt


@contextmanager
def precision(dt):
    prev = _compute_dtype
    set_compute_dtype(dt)
    try:
        yield
    finally:
        set_compute_dtype(prev)


def library_path():
    from ._lib import LIB_PATH
    return LIB_PATH


def load_library():
    from . import _lib
    return _lib.load()
