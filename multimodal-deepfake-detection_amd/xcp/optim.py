"""Fused gradient clipping + Adam for the training step (train_visual.py:575-577,
train_audio.py:40-44): ``clip_grad_norm_(params, max_norm)`` followed by
``torch.optim.Adam(params, lr, betas, eps, weight_decay)`` in two HIP launches over a chunk
table of every parameter (csrc/optim.hip), with the clip coefficient kept on the device.

Same update as torch's Adam (L2 weight decay, bias correction, no amsgrad).  Differences:
``param.grad`` keeps the unclipped gradient (clipping is applied inside the update), and
``step()`` returns the pre-clip total norm as a 0-d device tensor, as clip_grad_norm_ does.
"""
import math

import torch

from . import _lib, ops

CHUNK = 16384


class FusedAdamClip:
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0, max_norm=None):
        self.params = [p for p in params if p.requires_grad]
        for p in self.params:
            if p.dtype != torch.float32 or not p.is_contiguous():
                raise ValueError("FusedAdamClip: fp32 contiguous parameters only")
        ops.check_gpu(*self.params)
        self.lr, self.betas, self.eps, self.wd = lr, betas, eps, weight_decay
        self.max_norm = max_norm
        self.t = 0
        self.exp_avg = [torch.zeros_like(p) for p in self.params]
        self.exp_avg_sq = [torch.zeros_like(p) for p in self.params]
        dev = self.params[0].device
        self._out = torch.zeros(2, device=dev, dtype=torch.float32)
        self._key = None
        self._tab = None
        self._part = None

    def _table(self):
        key = tuple(p.grad.data_ptr() if p.grad is not None else 0 for p in self.params)
        if key != self._key:
            rows = []
            for p, m, v in zip(self.params, self.exp_avg, self.exp_avg_sq):
                if p.grad is None:
                    continue
                g = p.grad
                if g.dtype != torch.float32 or not g.is_contiguous():
                    raise ValueError("FusedAdamClip: fp32 contiguous gradients only")
                n = p.numel()
                for s in range(0, n, CHUNK):
                    rows.append([p.data_ptr(), g.data_ptr(), m.data_ptr(), v.data_ptr(), s, min(CHUNK, n - s)])
            self._tab = torch.tensor(rows, dtype=torch.int64).to(self.params[0].device)
            self._part = torch.empty(len(rows), device=self.params[0].device, dtype=torch.float32)
            self._key = key
        return self._tab

    @torch.no_grad()
    def step(self):
        tab = self._table()
        n = tab.shape[0]
        s = ops.stream()
        coef = 0
        if self.max_norm is not None:
            _lib.call("xcp_opt_sumsq", tab.data_ptr(), n, self._part.data_ptr(), float(self.max_norm),
                      self._out.data_ptr(), s)
            coef = self._out.data_ptr()
        self.t += 1
        b1, b2 = self.betas
        _lib.call("xcp_opt_adam", tab.data_ptr(), n, coef, float(self.lr), float(b1), float(b2), float(self.eps),
                  float(self.wd), float(1.0 - b1 ** self.t), float(math.sqrt(1.0 - b2 ** self.t)), s)
        return self._out[1]
