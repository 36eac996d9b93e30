"""PyTorch custom operators (namespace ``xcp``) over the C ABI: the module-level boundary.

The reference runs its Xception graph module by module through ATen (``SeparableConv2d``
Xception.py:37-47, ``Block`` :50-99, ``nn.BatchNorm2d``, ``nn.MaxPool2d``, ``nn.LSTM``).
These ``torch.library`` ops give the same per-module granularity on the gfx950 kernels, so
``model.block4(x)``, forward hooks on sub-modules and per-block probing work as in the
reference; the fused whole-backbone engine (xcp.engine) stays the fast path of
``Xception.forward``.

Every op:
  * has a fake (meta) kernel, so shapes propagate under FakeTensorMode / torch.compile
    tracing and on the ``meta`` device;
  * runs only on the GPU (a CPU tensor raises -- there is no CPU fallback);
  * computes in the dtype of its activation input (fp32 = parity mode, bf16 = throughput),
    with fp32 parameters and fp32 parameter gradients;
  * takes NCHW tensors and returns NCHW-shaped tensors in ``torch.channels_last`` memory
    (the kernels' NHWC "pixel rows"), so consecutive ops never transpose;
  * enters the tensor's device (ops.device_guard) and launches on its current stream.

Autograd is registered with ``register_autograd``; each backward is itself an ``xcp`` op.
"""
from typing import List, Optional, Tuple

import torch
from torch import Tensor

from . import ops
from .ops import ACT_NONE

CL = torch.channels_last


def _cl(x):
    ops.check_gpu(x)
    return x.contiguous(memory_format=CL)


def _nchw_like(N, C, H, W, x, dtype=None):
    return torch.empty((N, C, H, W), device=x.device, dtype=dtype or x.dtype, memory_format=CL)


def _stats(C, dev):
    from .engine import Stats
    return Stats(C, dev)


# ------------------------------------------------------------------ depthwise 3x3
@torch.library.custom_op("xcp::dwconv3x3", mutates_args=(), device_types="cuda")
def dwconv3x3(x: Tensor, weight: Tensor) -> Tensor:
    """nn.Conv2d(C, C, 3, 1, 1, groups=C, bias=False) (SeparableConv2d.conv1, Xception.py:41)."""
    with ops.device_guard(x):
        xc = _cl(x)
        N, C, H, W = xc.shape
        wt = weight.detach().float().reshape(C, 9).t().contiguous()
        y = _nchw_like(N, C, H, W, xc)
        ops.dw_fwd(ACT_NONE, xc, y, wt, None, None, N, H, W, C)
        return y


@dwconv3x3.register_fake
def _(x, weight):
    return torch.empty_like(x, memory_format=CL)


@torch.library.custom_op("xcp::dwconv3x3_backward", mutates_args=(), device_types="cuda")
def dwconv3x3_backward(grad: Tensor, x: Tensor, weight: Tensor) -> Tuple[Tensor, Tensor]:
    with ops.device_guard(x):
        xc, gc = _cl(x), _cl(grad).to(x.dtype)
        N, C, H, W = xc.shape
        wt = weight.detach().float().reshape(C, 9).t().contiguous()
        dx = _nchw_like(N, C, H, W, xc)
        dw = torch.empty((C, 1, 3, 3), device=x.device, dtype=torch.float32)
        ops.dw_bwd(ACT_NONE, gc, xc, wt, None, None, dx, dw, N, H, W, C)
        return dx, dw


@dwconv3x3_backward.register_fake
def _(grad, x, weight):
    return torch.empty_like(x, memory_format=CL), torch.empty(weight.shape, device=x.device, dtype=torch.float32)


def _dw_setup(ctx, inputs, output):
    ctx.save_for_backward(*inputs)


def _dw_bwd(ctx, grad):
    x, w = ctx.saved_tensors
    dx, dw = torch.ops.xcp.dwconv3x3_backward(grad, x, w)
    return dx, dw.to(w.dtype)


dwconv3x3.register_autograd(_dw_bwd, setup_context=_dw_setup)


# ------------------------------------------------------------------ pointwise 1x1 (stride s)
def _pw_geom(x, stride):
    N, C, H, W = x.shape
    OH, OW = (H - 1) // stride + 1, (W - 1) // stride + 1
    return N, C, H, W, OH, OW


@torch.library.custom_op("xcp::pointwise", mutates_args=(), device_types="cuda")
def pointwise(x: Tensor, weight: Tensor, stride: int) -> Tensor:
    """nn.Conv2d(Cin, Cout, 1, stride, bias=False): SeparableConv2d.pointwise (Xception.py:42) and
    Block.skip (Xception.py:55, stride 2) -- the MFMA GEMM Y[M, Cout] = X[M, Cin] W^T with a
    strided row gather."""
    with ops.device_guard(x):
        xc = _cl(x)
        N, C, H, W, OH, OW = _pw_geom(xc, stride)
        Cout = weight.shape[0]
        wp = weight.detach().reshape(Cout, C).to(xc.dtype).contiguous()
        y = _nchw_like(N, Cout, OH, OW, xc)
        gather = (1, H, W, OH, OW, stride, 0) if stride != 1 else (0, 0, 0, 0, 0, 1, 0)
        ops.gemm_nt(xc, wp, y, N * OH * OW, Cout, C, lda=C, gather=gather)
        return y


@pointwise.register_fake
def _(x, weight, stride):
    N, C, H, W, OH, OW = _pw_geom(x, stride)
    return torch.empty((N, weight.shape[0], OH, OW), device=x.device, dtype=x.dtype, memory_format=CL)


@torch.library.custom_op("xcp::pointwise_backward", mutates_args=(), device_types="cuda")
def pointwise_backward(grad: Tensor, x: Tensor, weight: Tensor, stride: int) -> Tuple[Tensor, Tensor]:
    with ops.device_guard(x):
        xc, gc = _cl(x), _cl(grad).to(x.dtype)
        N, C, H, W, OH, OW = _pw_geom(xc, stride)
        Cout = weight.shape[0]
        M = N * OH * OW
        wT = weight.detach().reshape(Cout, C).t().to(xc.dtype).contiguous()   # [Cin][Cout]
        if stride == 1:
            dx = _nchw_like(N, C, H, W, xc)
            ops.gemm_nt(gc, wT, dx, M, C, Cout)
        else:   # the strided conv's input gradient lives on the stride lattice
            dxs = _nchw_like(N, C, OH, OW, xc)
            ops.gemm_nt(gc, wT, dxs, M, C, Cout)
            dx = torch.empty((N, C, H, W), device=x.device, dtype=xc.dtype, memory_format=CL).zero_()
            dx[:, :, ::stride, ::stride] = dxs
        dw = torch.empty((Cout, C, 1, 1), device=x.device, dtype=torch.float32)
        gather = (1, H, W, OH, OW, stride, 0) if stride != 1 else (0, 0, 0, 0, 0, 1, 0)
        ops.weight_grad(gc, xc, M, Cout, C, dw, gather=gather, ldx=C)
        return dx, dw


@pointwise_backward.register_fake
def _(grad, x, weight, stride):
    return torch.empty_like(x, memory_format=CL), torch.empty(weight.shape, device=x.device, dtype=torch.float32)


def _pw_setup(ctx, inputs, output):
    x, w, stride = inputs
    ctx.save_for_backward(x, w)
    ctx.stride = stride


def _pw_bwd(ctx, grad):
    x, w = ctx.saved_tensors
    dx, dw = torch.ops.xcp.pointwise_backward(grad, x, w, ctx.stride)
    return dx, dw.to(w.dtype), None


pointwise.register_autograd(_pw_bwd, setup_context=_pw_setup)


# ------------------------------------------------------------------ BatchNorm2d
def _bn_ref(weight, bias, rm, rv, momentum, eps):
    return {"weight": weight, "bias": bias, "running_mean": rm, "running_var": rv, "eps": eps,
            "momentum": momentum, "track": rm is not None}


@torch.library.custom_op("xcp::batch_norm", mutates_args=(), device_types="cuda")
def batch_norm(x: Tensor, weight: Tensor, bias: Tensor, running_mean: Optional[Tensor], running_var: Optional[Tensor],
               training: bool, momentum: float, eps: float) -> Tuple[Tensor, Tensor, Tensor, Tensor, Tensor]:
    """nn.BatchNorm2d forward (Xception.py:56,67,73,78,119,123,143,147): training = batch
    statistics (biased variance to normalise, fp64 finalisation), else the running statistics.
    Functional: returns (y, mean, invstd, new running_mean, new running_var) -- in training
    the running statistics updated with momentum and the unbiased variance, as PyTorch does
    (empty tensors when running statistics are not tracked); xcp.modules.BatchNorm2d copies
    them into its buffers."""
    with ops.device_guard(x):
        xc = _cl(x)
        N, C, H, W = xc.shape
        rows = N * H * W
        rm = running_mean.detach().clone() if running_mean is not None else None
        rv = running_var.detach().clone() if running_var is not None else None
        bn = _bn_ref(weight.detach(), bias.detach(), rm, rv, momentum, eps)
        st = _stats(C, x.device)
        if training:
            part, R = ops.row_stats(xc, rows, C)
            ops.finalize_stats(part, R, C, rows, bn, True, st)   # updates rm / rv (the copies) in place
        else:
            ops.eval_stats(C, bn, st, x.device)
        y = _nchw_like(N, C, H, W, xc)
        ops.bn_act(xc, y, st.scale, st.shift, False, rows, C)
        empty = x.new_empty(0, dtype=torch.float32)
        return (y, st.mean.clone(), st.invstd.clone(), rm if rm is not None else empty,
                rv if rv is not None else empty.clone())


@batch_norm.register_fake
def _(x, weight, bias, running_mean, running_var, training, momentum, eps):
    C = x.shape[1]
    f = dict(dtype=torch.float32)
    return (torch.empty_like(x, memory_format=CL), x.new_empty(C, **f), x.new_empty(C, **f),
            x.new_empty(C if running_mean is not None else 0, **f), x.new_empty(C if running_var is not None else 0, **f))


@torch.library.custom_op("xcp::batch_norm_backward", mutates_args=(), device_types="cuda")
def batch_norm_backward(grad: Tensor, x: Tensor, weight: Tensor, mean: Tensor, invstd: Tensor,
                        training: bool) -> Tuple[Tensor, Tensor, Tensor]:
    with ops.device_guard(x):
        xc, gc = _cl(x), _cl(grad).to(x.dtype)
        N, C, H, W = xc.shape
        rows = N * H * W
        dx = _nchw_like(N, C, H, W, xc)
        dg = torch.empty(C, device=x.device, dtype=torch.float32)
        db = torch.empty(C, device=x.device, dtype=torch.float32)
        st = {"mean": mean, "invstd": invstd}
        if training:
            ops.bn_backward(gc, xc, rows, C, {"weight": weight.detach().float()}, st, dx, dg, db)
        else:
            # running statistics are constants: dx = dy * gamma * invstd (an affine map: the bn_act
            # kernel with scale = gamma * invstd, shift = 0), dgamma / dbeta from the BN reduce
            P = ops._lib.call("xcp_chanred_parts", rows, C)
            p = torch.empty(P * 2 * C, device=x.device, dtype=torch.float32)
            ops._lib.call("xcp_bn_bwd_reduce", ops.DT[xc.dtype], gc.data_ptr(), xc.data_ptr(), mean.data_ptr(),
                          invstd.data_ptr(), 0, 0, rows, C, p.data_ptr(), ops.stream())
            s = torch.empty(2 * C, device=x.device, dtype=torch.float32)
            ops.reduce_slabs(p, P, 2 * C, s)   # colreduce: fp64 sums over the partial rows
            db.copy_(s[:C])
            dg.copy_(s[C:])
            scale = (weight.detach().float() * invstd).contiguous()
            ops.bn_act(gc, dx, scale, torch.zeros_like(scale), False, rows, C)
        return dx, dg, db


@batch_norm_backward.register_fake
def _(grad, x, weight, mean, invstd, training):
    C = x.shape[1]
    return (torch.empty_like(x, memory_format=CL), x.new_empty(C, dtype=torch.float32),
            x.new_empty(C, dtype=torch.float32))


def _bn_setup(ctx, inputs, output):
    x, weight, bias, rm, rv, training, momentum, eps = inputs
    y, mean, invstd, nrm, nrv = output
    ctx.save_for_backward(x, weight, mean, invstd)
    ctx.training = training
    ctx.mark_non_differentiable(mean, invstd, nrm, nrv)


def _bn_bwd(ctx, grad, gmean, ginvstd, grm, grv):
    x, weight, mean, invstd = ctx.saved_tensors
    dx, dg, db = torch.ops.xcp.batch_norm_backward(grad, x, weight, mean, invstd, ctx.training)
    return dx, dg.to(weight.dtype), db.to(weight.dtype), None, None, None, None, None


batch_norm.register_autograd(_bn_bwd, setup_context=_bn_setup)


# ------------------------------------------------------------------ MaxPool2d(3, 2, 1)
@torch.library.custom_op("xcp::max_pool3x3s2", mutates_args=(), device_types="cuda")
def max_pool3x3s2(x: Tensor) -> Tuple[Tensor, Tensor]:
    """nn.MaxPool2d(3, 2, 1) (Block.rep, Xception.py:85-86) -> (y, argmax taps [N*OH*OW*C] uint8)."""
    with ops.device_guard(x):
        xc = _cl(x)
        N, C, H, W = xc.shape
        OH, OW = (H - 1) // 2 + 1, (W - 1) // 2 + 1
        one = torch.ones(C, device=x.device, dtype=torch.float32)
        zero = torch.zeros(C, device=x.device, dtype=torch.float32)
        skip = torch.zeros((N * OH * OW, C), device=x.device, dtype=xc.dtype)   # the tail kernel adds a skip term
        y = _nchw_like(N, C, OH, OW, xc)
        amax = torch.empty(N * OH * OW * C, device=x.device, dtype=torch.uint8)
        ops.tail_fwd(xc, one, zero, True, skip, None, None, y, amax, N, H, W, C)
        return y, amax


@max_pool3x3s2.register_fake
def _(x):
    N, C, H, W = x.shape
    OH, OW = (H - 1) // 2 + 1, (W - 1) // 2 + 1
    return (torch.empty((N, C, OH, OW), device=x.device, dtype=x.dtype, memory_format=CL),
            torch.empty(N * OH * OW * C, device=x.device, dtype=torch.uint8))


@torch.library.custom_op("xcp::max_pool3x3s2_backward", mutates_args=(), device_types="cuda")
def max_pool3x3s2_backward(grad: Tensor, amax: Tensor, H: int, W: int) -> Tensor:
    with ops.device_guard(grad):
        gc = _cl(grad)
        N, C = gc.shape[:2]
        dx = _nchw_like(N, C, H, W, gc)
        ops.maxpool_bwd(gc, amax, dx, N, H, W, C)
        return dx


@max_pool3x3s2_backward.register_fake
def _(grad, amax, H, W):
    N, C = grad.shape[:2]
    return torch.empty((N, C, H, W), device=grad.device, dtype=grad.dtype, memory_format=CL)


def _mp_setup(ctx, inputs, output):
    (x,) = inputs
    ctx.hw = x.shape[2:]
    ctx.save_for_backward(output[1])
    ctx.mark_non_differentiable(output[1])


def _mp_bwd(ctx, grad, gamax):
    (amax,) = ctx.saved_tensors
    return torch.ops.xcp.max_pool3x3s2_backward(grad, amax, ctx.hw[0], ctx.hw[1])


max_pool3x3s2.register_autograd(_mp_bwd, setup_context=_mp_setup)


# ------------------------------------------------------------------ stem convs
@torch.library.custom_op("xcp::stem_conv1", mutates_args=(), device_types="cuda")
def stem_conv1(x: Tensor, weight: Tensor, out_bf16: bool) -> Tensor:
    """Xception.conv1 = nn.Conv2d(3, 32, 3, 2, 0) (Xception.py:118) on fp32 NCHW input."""
    with ops.device_guard(x):
        ops.check_gpu(x)
        xc = x.float().contiguous()
        N, _, IH, IW = xc.shape
        OH, OW = (IH - 3) // 2 + 1, (IW - 3) // 2 + 1
        y = _nchw_like(N, 32, OH, OW, xc, torch.bfloat16 if out_bf16 else torch.float32)
        ops.conv1_fwd(xc, weight.detach().float().contiguous(), y, N, IH, IW)
        return y


@stem_conv1.register_fake
def _(x, weight, out_bf16):
    N, _, IH, IW = x.shape
    return torch.empty((N, 32, (IH - 3) // 2 + 1, (IW - 3) // 2 + 1), device=x.device,
                       dtype=torch.bfloat16 if out_bf16 else torch.float32, memory_format=CL)


@torch.library.custom_op("xcp::stem_conv1_wgrad", mutates_args=(), device_types="cuda")
def stem_conv1_wgrad(grad: Tensor, x: Tensor) -> Tensor:
    with ops.device_guard(x):
        xc = x.float().contiguous()
        N, _, IH, IW = xc.shape
        dw = torch.empty((32, 3, 3, 3), device=x.device, dtype=torch.float32)
        ops.conv1_wgrad(xc, _cl(grad), dw, N, IH, IW)
        return dw


@stem_conv1_wgrad.register_fake
def _(grad, x):
    return torch.empty((32, 3, 3, 3), device=x.device, dtype=torch.float32)


def _c1_setup(ctx, inputs, output):
    x, w, _ = inputs
    ctx.save_for_backward(x)


def _c1_bwd(ctx, grad):
    (x,) = ctx.saved_tensors
    if ctx.needs_input_grad[0]:
        raise NotImplementedError("xcp::stem_conv1: no gradient w.r.t. the input frames (the reference never "
                                  "differentiates w.r.t. its clips)")
    return None, torch.ops.xcp.stem_conv1_wgrad(grad, x), None


stem_conv1.register_autograd(_c1_bwd, setup_context=_c1_setup)


@torch.library.custom_op("xcp::stem_conv2", mutates_args=(), device_types="cuda")
def stem_conv2(x: Tensor, weight: Tensor) -> Tensor:
    """Xception.conv2 = nn.Conv2d(32, 64, 3) (Xception.py:122) as an implicit GEMM (im2col gather)."""
    with ops.device_guard(x):
        xc = _cl(x)
        N, C, H, W = xc.shape
        OH, OW = H - 2, W - 2
        wp = weight.detach().permute(0, 2, 3, 1).reshape(64, 9 * C).to(xc.dtype).contiguous()   # [co][tap][ci]
        y = _nchw_like(N, 64, OH, OW, xc)
        ops.gemm_nt(xc, wp, y, N * OH * OW, 64, 9 * C, lda=C, gather=(2, H, W, OH, OW, 1, C))
        return y


@stem_conv2.register_fake
def _(x, weight):
    N, C, H, W = x.shape
    return torch.empty((N, 64, H - 2, W - 2), device=x.device, dtype=x.dtype, memory_format=CL)


@torch.library.custom_op("xcp::stem_conv2_backward", mutates_args=(), device_types="cuda")
def stem_conv2_backward(grad: Tensor, x: Tensor, weight: Tensor) -> Tuple[Tensor, Tensor]:
    with ops.device_guard(x):
        xc, gc = _cl(x), _cl(grad).to(x.dtype)
        N, C, H, W = xc.shape
        OH, OW = H - 2, W - 2
        wt = weight.detach().permute(1, 2, 3, 0).reshape(C, 9 * 64).to(xc.dtype).contiguous()   # [ci][tap][co]
        dx = _nchw_like(N, C, H, W, xc)
        ops.gemm_nt(gc, wt, dx, N * H * W, C, 9 * 64, lda=64, gather=(3, H, W, OH, OW, 1, 64))
        wg = torch.empty(64 * 9 * C, device=x.device, dtype=torch.float32)
        ops.weight_grad(gc, xc, N * OH * OW, 64, 9 * C, wg, gather=(2, H, W, OH, OW, 1, C), ldx=C)
        return dx, wg.view(64, 3, 3, C).permute(0, 3, 1, 2).contiguous()


@stem_conv2_backward.register_fake
def _(grad, x, weight):
    return torch.empty_like(x, memory_format=CL), torch.empty(weight.shape, device=x.device, dtype=torch.float32)


def _c2_setup(ctx, inputs, output):
    ctx.save_for_backward(*inputs)


def _c2_bwd(ctx, grad):
    x, w = ctx.saved_tensors
    dx, dw = torch.ops.xcp.stem_conv2_backward(grad, x, w)
    return dx, dw.to(w.dtype)


stem_conv2.register_autograd(_c2_bwd, setup_context=_c2_setup)


# ------------------------------------------------------------------ LSTM (nn.LSTM, 1 layer, batch_first)
@torch.library.custom_op("xcp::lstm", mutates_args=(), device_types="cuda")
def lstm(x: Tensor, w_ih: Tensor, w_hh: Tensor, b_ih: Tensor, b_hh: Tensor,
         kernel: int) -> Tuple[Tensor, Tensor, Tensor, Tensor, Tensor, Tensor]:
    """nn.LSTM(I, H, 1, batch_first=True) forward (XceptionLSTMV.py:18-23, :67; gates i, f, g, o;
    h0 = c0 = 0): the input projection of all T steps is one fp32 MFMA GEMM, the recurrence one
    fused kernel per time direction (lstm.hip).  Returns (out [B,T,H], h_n [1,B,H], c_n [1,B,H]) and
    the saved state (h_{t-1}, c_t [B,T,H], activated gates [B,T,4H]) for the backward."""
    with ops.device_guard(x):
        ops.check_gpu(x, w_ih)
        B, T, I = x.shape
        H = w_hh.shape[1]
        dev = x.device
        xf = x.detach().float().contiguous()
        xproj = torch.empty(B * T, 4 * H, device=dev, dtype=torch.float32)
        ops.gemm_nt(xf, w_ih.detach().float().contiguous(), xproj, B * T, 4 * H, I)
        whh = w_hh.detach().float().contiguous()
        whhT = None
        if ops.lstm_needs_whhT(B, H, kernel):
            whhT = torch.empty(H * 4 * H, device=dev, dtype=torch.float32)
            ops.permute3(whh, whhT, 4 * H, H, 1, (1, 0, 2))
        out = torch.empty(B, T, H, device=dev, dtype=torch.float32)
        hprev = torch.empty(B, T, H, device=dev, dtype=torch.float32)
        cst = torch.empty(B, T, H, device=dev, dtype=torch.float32)
        gates = torch.empty(B, T, 4 * H, device=dev, dtype=torch.float32)
        hn = torch.empty(1, B, H, device=dev, dtype=torch.float32)
        cn = torch.empty(1, B, H, device=dev, dtype=torch.float32)
        ops.lstm_fwd(xproj, whh, whhT, b_ih.detach().float().contiguous(), b_hh.detach().float().contiguous(), out,
                     hprev, cst, gates, hn, cn, B, T, H, kernel)
        return out, hn, cn, hprev, cst, gates


@lstm.register_fake
def _(x, w_ih, w_hh, b_ih, b_hh, kernel):
    B, T, _ = x.shape
    H = w_hh.shape[1]
    f = dict(device=x.device, dtype=torch.float32)
    return (torch.empty(B, T, H, **f), torch.empty(1, B, H, **f), torch.empty(1, B, H, **f), torch.empty(B, T, H, **f),
            torch.empty(B, T, H, **f), torch.empty(B, T, 4 * H, **f))


@torch.library.custom_op("xcp::lstm_backward", mutates_args=(), device_types="cuda")
def lstm_backward(dout: Optional[Tensor], dhn: Optional[Tensor], dcn: Optional[Tensor], x: Tensor, w_ih: Tensor,
                  w_hh: Tensor, hprev: Tensor, cst: Tensor, gates: Tensor, kernel: int,
                  need_dx: bool) -> Tuple[Tensor, Tensor, Tensor, Tensor]:
    with ops.device_guard(x):
        B, T, I = x.shape
        H = w_hh.shape[1]
        dev = x.device
        M = B * T
        xf = x.detach().float().contiguous()
        dgates = torch.empty(M, 4 * H, device=dev, dtype=torch.float32)
        f32 = lambda t: None if t is None else t.float().contiguous()   # noqa: E731
        ops.lstm_bwd(f32(dout), f32(dhn), f32(dcn), w_hh.detach().float().contiguous(), cst, gates, dgates, B, T, H,
                     kernel)
        dw_ih = torch.empty(4 * H, I, device=dev, dtype=torch.float32)
        ops.weight_grad(dgates, xf, M, 4 * H, I, dw_ih)
        dw_hh = torch.empty(4 * H, H, device=dev, dtype=torch.float32)
        ops.weight_grad(dgates, hprev, M, 4 * H, H, dw_hh)
        db = torch.empty(4 * H, device=dev, dtype=torch.float32)
        ops.reduce_slabs(dgates, M, 4 * H, db)
        if need_dx:
            wT = torch.empty(I * 4 * H, device=dev, dtype=torch.float32)
            ops.permute3(w_ih.detach().float().contiguous(), wT, 4 * H, I, 1, (1, 0, 2))
            dx = torch.empty(B, T, I, device=dev, dtype=torch.float32)
            ops.gemm_nt(dgates, wT, dx, M, I, 4 * H)
        else:
            dx = torch.empty(0, device=dev, dtype=torch.float32)
        return dx, dw_ih, dw_hh, db


@lstm_backward.register_fake
def _(dout, dhn, dcn, x, w_ih, w_hh, hprev, cst, gates, kernel, need_dx):
    B, T, I = x.shape
    f = dict(device=x.device, dtype=torch.float32)
    return (torch.empty(B, T, I, **f) if need_dx else torch.empty(0, **f), torch.empty(w_ih.shape, **f),
            torch.empty(w_hh.shape, **f), torch.empty(w_ih.shape[0], **f))


def _lstm_setup(ctx, inputs, output):
    x, w_ih, w_hh, b_ih, b_hh, kernel = inputs
    out, hn, cn, hprev, cst, gates = output
    ctx.save_for_backward(x, w_ih, w_hh, hprev, cst, gates)
    ctx.kernel = kernel
    ctx.x_dtype = x.dtype
    ctx.mark_non_differentiable(hprev, cst, gates)


def _lstm_bwd(ctx, dout, dhn, dcn, *_):
    x, w_ih, w_hh, hprev, cst, gates = ctx.saved_tensors
    need_dx = ctx.needs_input_grad[0]
    dx, dw_ih, dw_hh, db = torch.ops.xcp.lstm_backward(dout, dhn, dcn, x, w_ih, w_hh, hprev, cst, gates, ctx.kernel,
                                                       need_dx)
    return (dx.to(ctx.x_dtype) if need_dx else None, dw_ih, dw_hh, db, db.clone(), None)


lstm.register_autograd(_lstm_bwd, setup_context=_lstm_setup)


OPS: List[str] = ["dwconv3x3", "dwconv3x3_backward", "pointwise", "pointwise_backward", "batch_norm",
                  "batch_norm_backward", "max_pool3x3s2", "max_pool3x3s2_backward", "stem_conv1", "stem_conv1_wgrad",
                  "stem_conv2", "stem_conv2_backward", "lstm", "lstm_backward"]
