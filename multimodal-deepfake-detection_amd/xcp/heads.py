"""Classification heads and losses of the reference's training scripts, on HIP kernels
(csrc/heads.hip) behind ``torch.library`` ops ``xcp::arcface`` and ``xcp::focal_ce``.

* ``ArcFaceHead`` -- train_visual.py:455-474 (s = 30, m = 0.5, used with CrossEntropyLoss,
  :527-531, :570-572) and train_au_face.py:423-442 (m = 0.30).  Same constructor, parameter
  (``weight`` [num_classes, feat_dim]), init (``torch.randn`` then ``xavier_uniform_``: the same
  RNG draws) and ``state_dict``; ``forward(features, labels=None)`` as the reference's.
* ``CBFocalLoss`` -- train_au_face.py:445-458 (class-balanced weights from samples per
  class, beta 0.9999, gamma 2), as the reference's, including the ``class_weights`` buffer.
* ``cross_entropy`` -- the mean cross entropy of train_visual.py:527 on the same kernel.

Inputs of any float dtype (e.g. fp16 under autocast) are computed in fp32; the outputs are
fp32.  Both ops run on the GPU only.
"""
from typing import Optional, Tuple

import numpy as np
import torch
import torch.nn as nn
from torch import Tensor

from . import _lib, ops


def _p(t):
    return 0 if t is None else t.data_ptr()


@torch.library.custom_op("xcp::arcface", mutates_args=(), device_types="cuda")
def arcface(features: Tensor, weight: Tensor, labels: Optional[Tensor], s: float, m: float) -> Tensor:
    with ops.device_guard(features):
        ops.check_gpu(features, weight)
        x = features.detach().float().contiguous()
        W = weight.detach().float().contiguous()
        B, D = x.shape
        C = W.shape[0]
        lab = labels.long().contiguous() if labels is not None else None
        out = torch.empty(B, C, device=x.device, dtype=torch.float32)
        _lib.call("xcp_arcface_fwd", _p(x), _p(W), _p(lab), _p(out), B, C, D, float(s), float(m), ops.stream())
        return out


@arcface.register_fake
def _(features, weight, labels, s, m):
    return features.new_empty(features.shape[0], weight.shape[0], dtype=torch.float32)


@torch.library.custom_op("xcp::arcface_backward", mutates_args=(), device_types="cuda")
def arcface_backward(grad: Tensor, features: Tensor, weight: Tensor, labels: Optional[Tensor], s: float,
                     m: float) -> Tuple[Tensor, Tensor]:
    with ops.device_guard(features):
        x = features.detach().float().contiguous()
        W = weight.detach().float().contiguous()
        B, D = x.shape
        C = W.shape[0]
        lab = labels.long().contiguous() if labels is not None else None
        g = grad.float().contiguous()
        dx = torch.empty_like(x)
        dw = torch.empty_like(W)
        _lib.call("xcp_arcface_bwd", _p(x), _p(W), _p(lab), _p(g), _p(dx), _p(dw), B, C, D, float(s), float(m),
                  ops.stream())
        return dx, dw


@arcface_backward.register_fake
def _(grad, features, weight, labels, s, m):
    return features.new_empty(features.shape, dtype=torch.float32), weight.new_empty(weight.shape, dtype=torch.float32)


def _af_setup(ctx, inputs, output):
    features, weight, labels, s, m = inputs
    ctx.save_for_backward(features, weight, labels)
    ctx.sm = (s, m)


def _af_bwd(ctx, grad):
    features, weight, labels = ctx.saved_tensors
    dx, dw = torch.ops.xcp.arcface_backward(grad, features, weight, labels, *ctx.sm)
    return dx.to(features.dtype), dw.to(weight.dtype), None, None, None


arcface.register_autograd(_af_bwd, setup_context=_af_setup)


@torch.library.custom_op("xcp::focal_ce", mutates_args=(), device_types="cuda")
def focal_ce(logits: Tensor, labels: Tensor, weights: Optional[Tensor], gamma: float) -> Tensor:
    """mean_i (1 - pt_i)^gamma ce_i, ce_i = w[y_i] (logsumexp(z_i) - z_i[y_i]), pt = exp(-ce)."""
    with ops.device_guard(logits):
        ops.check_gpu(logits, labels)
        z = logits.detach().float().contiguous()
        B, C = z.shape
        w = weights.float().contiguous() if weights is not None else None
        loss = torch.empty((), device=z.device, dtype=torch.float32)
        _lib.call("xcp_focal_ce", _p(z), _p(labels.long().contiguous()), _p(w), float(gamma), 0, _p(loss), 0, B, C,
                  ops.stream())
        return loss


@focal_ce.register_fake
def _(logits, labels, weights, gamma):
    return logits.new_empty((), dtype=torch.float32)


@torch.library.custom_op("xcp::focal_ce_backward", mutates_args=(), device_types="cuda")
def focal_ce_backward(grad: Tensor, logits: Tensor, labels: Tensor, weights: Optional[Tensor], gamma: float) -> Tensor:
    with ops.device_guard(logits):
        z = logits.detach().float().contiguous()
        B, C = z.shape
        w = weights.float().contiguous() if weights is not None else None
        g = grad.float().contiguous()
        dz = torch.empty_like(z)
        scratch = torch.empty((), device=z.device, dtype=torch.float32)
        _lib.call("xcp_focal_ce", _p(z), _p(labels.long().contiguous()), _p(w), float(gamma), _p(g), _p(scratch),
                  _p(dz), B, C, ops.stream())
        return dz


@focal_ce_backward.register_fake
def _(grad, logits, labels, weights, gamma):
    return logits.new_empty(logits.shape, dtype=torch.float32)


def _fc_setup(ctx, inputs, output):
    logits, labels, weights, gamma = inputs
    ctx.save_for_backward(logits, labels, weights)
    ctx.gamma = gamma


def _fc_bwd(ctx, grad):
    logits, labels, weights = ctx.saved_tensors
    dz = torch.ops.xcp.focal_ce_backward(grad, logits, labels, weights, ctx.gamma)
    return dz.to(logits.dtype), None, None, None


focal_ce.register_autograd(_fc_bwd, setup_context=_fc_setup)


class ArcFaceHead(nn.Module):
    """ArcFace margin head (train_visual.py:455-474 with m = 0.5; train_au_face.py:423-442
    with m = 0.30)."""

    def __init__(self, feat_dim, num_classes=2, s=30.0, m=0.5):
        super().__init__()
        self.num_classes = num_classes
        self.s = s
        self.m = m
        self.weight = nn.Parameter(torch.randn(num_classes, feat_dim))
        nn.init.xavier_uniform_(self.weight)

    def forward(self, features, labels=None):
        return torch.ops.xcp.arcface(features, self.weight, labels, float(self.s), float(self.m))


class CBFocalLoss(nn.Module):
    """Class-Balanced Focal Loss on logits (train_au_face.py:445-458)."""

    def __init__(self, samples_per_cls, beta=0.9999, gamma=2.0):
        super().__init__()
        effective_num = 1.0 - np.power(beta, samples_per_cls)
        weights = (1.0 - beta) / np.array(effective_num)
        weights = weights / weights.sum() * len(samples_per_cls)
        self.register_buffer("class_weights", torch.tensor(weights, dtype=torch.float32))
        self.gamma = gamma

    def forward(self, logits, labels):
        return torch.ops.xcp.focal_ce(logits, labels, self.class_weights, float(self.gamma))


def cross_entropy(logits, labels):
    """nn.CrossEntropyLoss()(logits, labels) (mean over the batch; train_visual.py:527, :572)."""
    return torch.ops.xcp.focal_ce(logits, labels, None, 0.0)
