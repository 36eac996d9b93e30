"""``nn.LSTM`` drop-in whose forward/backward run on the xcp kernels.

Reference: the single-layer, batch_first ``nn.LSTM(2048, H)`` of
XceptionLSTMV.py:18-23 / XceptionLSTMA.py:14-19, used as ``self.lstm(features)``
(XceptionLSTMV.py:67) and as ``model.lstm(features)[0][:, -1, :]``
(train_visual.py:569).  Subclassing ``nn.LSTM`` keeps the parameter names
(``weight_ih_l0`` ...), the init (uniform(-1/sqrt(H), 1/sqrt(H)), same RNG
consumption) and the state_dict, so reference checkpoints load unchanged.

The input projection for all T steps is one fp32 MFMA GEMM; the recurrence is
one fused kernel per direction of time (lstm.hip).  The head runs in fp32 in
every precision mode (it is ~0.1 GFLOP per clip).
"""
import torch
import torch.nn as nn

from . import ops


class LSTMFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w_ih, w_hh, b_ih, b_hh):
        ops.check_gpu(x, w_ih)
        B, T, I = x.shape
        H = w_hh.shape[1]
        dev = x.device
        xf = x.detach().float().contiguous()
        M = B * T
        xproj = torch.empty(M, 4 * H, device=dev, dtype=torch.float32)
        ops.gemm_nt(xf, w_ih.detach().contiguous(), xproj, M, 4 * H, I)
        whh = w_hh.detach().contiguous()
        whhT = None
        if ops.lstm_needs_whhT(H):
            whhT = torch.empty(H * 4 * H, device=dev, dtype=torch.float32)
            ops.permute3(whh, whhT, 4 * H, H, 1, (1, 0, 2))
        out = torch.empty(B, T, H, device=dev, dtype=torch.float32)
        hprev = torch.empty(B, T, H, device=dev, dtype=torch.float32)
        cst = torch.empty(B, T, H, device=dev, dtype=torch.float32)
        gates = torch.empty(B, T, 4 * H, device=dev, dtype=torch.float32)
        hn = torch.empty(1, B, H, device=dev, dtype=torch.float32)
        cn = torch.empty(1, B, H, device=dev, dtype=torch.float32)
        ops.lstm_fwd(xproj, whh, whhT, b_ih.detach(), b_hh.detach(), out, hprev, cst, gates, hn, cn, B, T, H)
        ctx.save_for_backward(xf, w_ih, w_hh, hprev, cst, gates)
        ctx.dims = (B, T, I, H)
        ctx.x_dtype = x.dtype
        return out, hn, cn

    @staticmethod
    def backward(ctx, dout, dhn, dcn):
        xf, w_ih, w_hh, hprev, cst, gates = ctx.saved_tensors
        B, T, I, H = ctx.dims
        dev = xf.device
        M = B * T
        dgates = torch.empty(M, 4 * H, device=dev, dtype=torch.float32)
        ops.lstm_bwd(None if dout is None else dout.float().contiguous(),
                     None if dhn is None else dhn.float().contiguous(),
                     None if dcn is None else dcn.float().contiguous(), w_hh.detach().contiguous(), cst, gates, dgates, B,
                     T, H)
        dw_ih = dw_hh = db = dx = None
        if ctx.needs_input_grad[1]:
            dw_ih = torch.empty(4 * H, I, device=dev, dtype=torch.float32)
            ops.weight_grad(dgates, xf, M, 4 * H, I, dw_ih)
        if ctx.needs_input_grad[2]:
            dw_hh = torch.empty(4 * H, H, device=dev, dtype=torch.float32)
            ops.weight_grad(dgates, hprev, M, 4 * H, H, dw_hh)
        if ctx.needs_input_grad[3] or ctx.needs_input_grad[4]:
            db = torch.empty(4 * H, device=dev, dtype=torch.float32)
            ops.reduce_slabs(dgates, M, 4 * H, db)
        if ctx.needs_input_grad[0]:
            wT = torch.empty(I * 4 * H, device=dev, dtype=torch.float32)
            ops.permute3(w_ih.detach().contiguous(), wT, 4 * H, I, 1, (1, 0, 2))
            dx = torch.empty(B, T, I, device=dev, dtype=torch.float32)
            ops.gemm_nt(dgates, wT, dx, M, I, 4 * H)
            dx = dx.to(ctx.x_dtype)
        return dx, dw_ih, dw_hh, db, (db.clone() if db is not None else None)


class LSTM(nn.LSTM):
    """nn.LSTM with the xcp forward.  Supported configuration (the reference's):
    num_layers=1, batch_first=True, unidirectional, bias=True, proj_size=0, no
    initial state."""

    def forward(self, input, hx=None):  # noqa: A002  (nn.LSTM signature)
        if (self.num_layers != 1 or not self.batch_first or self.bidirectional or not self.bias or self.proj_size
                or hx is not None):
            raise NotImplementedError("xcp LSTM supports the reference configuration only "
                                      "(1 layer, batch_first, unidirectional, bias, zero initial state)")
        if input.dim() != 3:
            raise NotImplementedError("xcp LSTM expects batched [B, T, F] input")
        out, hn, cn = LSTMFunction.apply(input, self.weight_ih_l0, self.weight_hh_l0, self.bias_ih_l0,
                                         self.bias_hh_l0)
        return out, (hn, cn)
