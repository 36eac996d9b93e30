"""xcp -- MI355X-native (gfx950 HIP) runtime for the Xception + LSTM clip path.

Layout:
  csrc/      hand-written HIP kernels + the C ABI (declared in include/xcp.h)
  build.py   hipcc build of the in-tree libxcp.so
  _lib.py    ctypes binding of the C ABI (fails loudly when the library is missing)
  ops.py     typed wrappers over torch device tensors
  engine.py  whole-backbone forward/backward executor + autograd node
  lstm.py    nn.LSTM drop-in on the fused LSTM kernels
  ddp.py     one-process-per-GPU data parallelism over RCCL

Precision: activations / GEMM operands are bf16 by default (fp32 accumulation,
fp32 master weights, fp64 BN statistics); ``set_compute_dtype(torch.float32)`` or
``XCP_DTYPE=fp32`` selects the fp32 parity mode.
"""
import os
from contextlib import contextmanager

import torch

_DTYPES = {"bf16": torch.bfloat16, "bfloat16": torch.bfloat16, "fp32": torch.float32, "float32": torch.float32}
_compute_dtype = _DTYPES[os.environ.get("XCP_DTYPE", "bf16").lower()]


def compute_dtype():
    return _compute_dtype


def set_compute_dtype(dt):
    global _compute_dtype
    if isinstance(dt, str):
        dt = _DTYPES[dt.lower()]
    if dt not in (torch.float32, torch.bfloat16):
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
