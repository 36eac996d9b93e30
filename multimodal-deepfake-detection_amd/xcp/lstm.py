"""``nn.LSTM`` drop-in whose forward/backward run on the xcp kernels.

Reference: the single-layer, batch_first ``nn.LSTM(2048, H)`` of
XceptionLSTMV.py:18-23 / XceptionLSTMA.py:14-19, used as ``self.lstm(features)``
(XceptionLSTMV.py:67) and as ``model.lstm(features)[0][:, -1, :]``
(train_visual.py:569).  Subclassing ``nn.LSTM`` keeps the parameter names
(``weight_ih_l0`` ...), the init (uniform(-1/sqrt(H), 1/sqrt(H)), same RNG
consumption) and the state_dict, so reference checkpoints load unchanged.

The computation is the ``torch.ops.xcp.lstm`` custom op (xcp/torch_ops.py): the input
projection for all T steps is one fp32 MFMA GEMM, the recurrence one fused kernel per
direction of time (lstm.hip).  The head runs in fp32 in every precision mode (it is
~0.1 GFLOP per clip).
"""
import torch
import torch.nn as nn

from . import torch_ops  # noqa: F401  (registers torch.ops.xcp.lstm)


class LSTM(nn.LSTM):
    """nn.LSTM with the xcp forward.  Supported configuration (the reference's):
    num_layers=1, batch_first=True, unidirectional, bias=True, proj_size=0, no
    initial state.  ``xcp_kernel`` (attribute): 0 = automatic recurrence kernel choice,
    1 = the generic kernels."""

    xcp_kernel = 0

    def forward(self, input, hx=None):  # noqa: A002  (nn.LSTM signature)
        if (self.num_layers != 1 or not self.batch_first or self.bidirectional or not self.bias or self.proj_size
                or hx is not None):
            raise NotImplementedError("xcp LSTM supports the reference configuration only "
                                      "(1 layer, batch_first, unidirectional, bias, zero initial state)")
        if input.dim() != 3:
            raise NotImplementedError("xcp LSTM expects batched [B, T, F] input")
        if not input.is_cuda:
            raise RuntimeError("xcp LSTM runs on the MI355X only (got a non-GPU tensor); there is no CPU fallback")
        out, hn, cn, _, _, _ = torch.ops.xcp.lstm(input, self.weight_ih_l0, self.weight_hh_l0, self.bias_ih_l0,
                                                  self.bias_hh_l0, int(self.xcp_kernel))
        return out.to(input.dtype), (hn, cn)
