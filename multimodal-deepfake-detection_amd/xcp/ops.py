"""Thin typed wrappers over the C ABI (include/xcp.h) taking torch device tensors.

Torch is used only as the device-memory / stream provider: every compute call
below launches a hand-written gfx950 kernel from ``libxcp.so`` on the current
HIP stream.  There is no CPU or eager-PyTorch fallback: a missing library or a
non-GPU tensor raises.
"""
import torch

from . import _lib

F32, BF16 = 0, 1
ACT_NONE, ACT_RELU, ACT_BNRELU = 0, 1, 2
DT = {torch.float32: F32, torch.bfloat16: BF16}


def _p(t):
    return 0 if t is None else t.data_ptr()


def stream():
    return torch.cuda.current_stream().cuda_stream


class KernelTimer:
    """Brackets selected kernel launches with HIP events on the stream they are
    launched on (the current stream), for per-launch durations inside a timed
    region.  ``classes``: name -> predicate(op_name, args_dict)."""

    def __init__(self, classes):
        self.classes = classes
        self.events = {k: [] for k in classes}

    def match(self, op, a):
        for k, pred in self.classes.items():
            if pred(op, a):
                return k
        return None

    def mean_ms(self, k):
        ev = self.events.get(k) or []
        if not ev:
            return None
        return sum(s.elapsed_time(e) for s, e in ev) / len(ev)

    def count(self, k):
        return len(self.events.get(k) or [])


_timer = None


def set_kernel_timer(t):
    global _timer
    _timer = t


class _timed:
    def __init__(self, op, a):
        self.key = _timer.match(op, a) if _timer is not None else None

    def __enter__(self):
        if self.key is not None:
            self.s = torch.cuda.Event(enable_timing=True)
            self.e = torch.cuda.Event(enable_timing=True)
            self.s.record()

    def __exit__(self, *exc):
        if self.key is not None:
            self.e.record()
            _timer.events[self.key].append((self.s, self.e))


def check_gpu(*ts):
    for t in ts:
        if t is not None and not t.is_cuda:
            raise RuntimeError("xcp ops run on the MI355X only (got a non-GPU tensor); there is no CPU fallback")


# ---------------------------------------------------------------- GEMM
def gemm_nt(A, B, C, M, N, K, lda=None, ldb=None, ldc=None, stats=None, gather=(0, 0, 0, 0, 0, 1, 0)):
    dt = DT[A.dtype]
    with _timed("gemm_nt", {"M": M, "N": N, "K": K, "stats": stats}):
        _lib.call("xcp_gemm_nt", dt, _p(A), lda or K, _p(B), ldb or K, _p(C), ldc or N, M, N, K, _p(stats), *gather,
                  stream())


def gemm_tn(G, X, P, M, N, K, S, rows_per_split, ldg=None, ldx=None, gather=(0, 0, 0, 0, 0, 1, 0)):
    dt = DT[G.dtype]
    _lib.call("xcp_gemm_tn", dt, _p(G), ldg or N, _p(X), ldx or K, _p(P), M, N, K, S, rows_per_split, *gather,
              stream())


def nt_stat_rows(M):
    return _lib.call("xcp_gemm_nt_stat_rows", M)


def colreduce_f64(inp, S, L, out, G):
    _lib.call("xcp_colreduce_f64", _p(inp), S, L, _p(out), G, stream())


def colreduce_f32(inp, S, L, out, G):
    _lib.call("xcp_colreduce_f32", _p(inp), S, L, _p(out), G, stream())


def reduce_slabs(P, S, L, out):
    """out[L] = sum_s P[s][L] (fp32, deterministic, two levels when S is large)."""
    if S > 64:
        g = 32
        tmp = torch.empty(g * L, device=P.device, dtype=torch.float32)
        colreduce_f32(P, S, L, tmp, g)
        colreduce_f32(tmp, g, L, out, 1)
    else:
        colreduce_f32(P, S, L, out, 1)


def weight_grad(G, X, M, N, K, out, gather=(0, 0, 0, 0, 0, 1, 0), ldg=None, ldx=None):
    """out[N][K] (fp32) = G[M][N]^T X[M][K]."""
    rps = _lib.call("xcp_gemm_tn_rows_per_split", DT[G.dtype], gather[0], M, N, K)
    S = (M + rps - 1) // rps
    P = torch.empty(S * N * K, device=G.device, dtype=torch.float32)
    gemm_tn(G, X, P, M, N, K, S, rps, ldg=ldg, ldx=ldx, gather=gather)
    reduce_slabs(P, S, N * K, out)


# ---------------------------------------------------------------- depthwise
def dw_fwd(act, X, Y, Wt, scale, shift, N, H, W, C):
    with _timed("dw_fwd", {"N": N, "H": H, "W": W, "C": C}):
        _lib.call("xcp_dw_fwd", DT[X.dtype], act, _p(X), _p(Y), _p(Wt), _p(scale), _p(shift), N, H, W, C, stream())


def dw_bwd(act, dY, X, Wt, scale, shift, dX, dW_out, N, H, W, C, dRes=None, dSkip=None, skip_geom=(0, 0, 1),
           bn_stats=None):
    """Returns (bnpart, P) -- the preceding BN's backward partial sums -- when bn_stats
    (that BN's Stats) is given, else (None, 0)."""
    P = _lib.call("xcp_dw_bwd_chunks", N, H, W, C)
    part = torch.empty(P * C * 9, device=dY.device, dtype=torch.float32)
    bnpart = None
    if bn_stats is not None:
        bnpart = torch.empty(P * 2 * C, device=dY.device, dtype=torch.float32)
    _lib.call("xcp_dw_bwd", DT[dY.dtype], act, _p(dY), _p(X), _p(Wt), _p(scale), _p(shift), _p(dRes), _p(dSkip),
              skip_geom[0], skip_geom[1], skip_geom[2], _p(dX), _p(part), _p(bnpart),
              _p(bn_stats["mean"]) if bn_stats is not None else 0,
              _p(bn_stats["invstd"]) if bn_stats is not None else 0, N, H, W, C, stream())
    reduce_slabs(part, P, C * 9, dW_out)
    return bnpart, (P if bnpart is not None else 0)


# ---------------------------------------------------------------- batchnorm
STAT_GROUPS = 64


def finalize_stats(part, R, C, count, bn, train, out):
    """part: fp32 [R][2][C] partial sums -> out dict of mean/invstd/scale/shift (fp32 [C]).
    Updates bn running stats in place when train."""
    dev = part.device
    G = min(STAT_GROUPS, R)
    p2 = torch.empty(G * 2 * C, device=dev, dtype=torch.float64)
    colreduce_f64(part, R, 2 * C, p2, G)
    _bn_finalize(p2, G, C, count, bn, train, out)


def _bn_finalize(p2, G, C, count, bn, train, out):
    mom = bn["momentum"]
    _lib.call("xcp_bn_finalize", _p(p2), G, C, float(count), _p(bn["weight"]), _p(bn["bias"]),
              _p(bn["running_mean"]) if (train and bn["track"]) or not train else 0,
              _p(bn["running_var"]) if (train and bn["track"]) or not train else 0, float(mom), float(bn["eps"]),
              1 if train else 0, _p(out["mean"]), _p(out["invstd"]), _p(out["scale"]), _p(out["shift"]), stream())


def eval_stats(C, bn, out, device):
    p2 = torch.zeros(2 * C, device=device, dtype=torch.float64)
    _bn_finalize(p2, 1, C, 1.0, bn, False, out)


def row_stats(X, rows, C):
    R = _lib.call("xcp_chanred_parts", rows, C)
    part = torch.empty(R * 2 * C, device=X.device, dtype=torch.float32)
    _lib.call("xcp_row_stats", DT[X.dtype], _p(X), rows, C, _p(part), stream())
    return part, R


def bn_backward(dZ, Y, rows, C, bn, st, dY, dgamma, dbeta, part=None, R=0):
    """dY = BatchNorm2d backward (train-mode batch stats) of dZ; writes dgamma/dbeta.
    ``part`` ([R][2][C] partial (sum dz, sum dz*zhat)) may come fused from the
    producer of dZ; otherwise it is reduced here."""
    if part is None:
        R = _lib.call("xcp_chanred_parts", rows, C)
        part = torch.empty(R * 2 * C, device=dZ.device, dtype=torch.float32)
        _lib.call("xcp_bn_bwd_reduce", DT[dZ.dtype], _p(dZ), _p(Y), _p(st["mean"]), _p(st["invstd"]), rows, C,
                  _p(part), stream())
    G = min(STAT_GROUPS, R)
    p2 = torch.empty(G * 2 * C, device=dZ.device, dtype=torch.float64)
    colreduce_f64(part, R, 2 * C, p2, G)
    coef = torch.empty(3 * C, device=dZ.device, dtype=torch.float32)
    _lib.call("xcp_bn_bwd_finalize", _p(p2), G, C, float(rows), _p(bn["weight"]), _p(st["mean"]), _p(st["invstd"]),
              _p(coef), _p(coef[C:]), _p(coef[2 * C:]), _p(dgamma), _p(dbeta), 0, stream())
    _lib.call("xcp_bn_bwd_apply", DT[dZ.dtype], _p(dZ), _p(Y), _p(dY), _p(coef), _p(coef[C:]), _p(coef[2 * C:]), rows,
              C, stream())


def bn_act(X, Y, scale, shift, relu, rows, C):
    _lib.call("xcp_bn_act", DT[X.dtype], _p(X), _p(Y), _p(scale), _p(shift), 1 if relu else 0, rows, C, stream())


def relu_bwd(dX, X, rows, C):
    _lib.call("xcp_relu_bwd", DT[dX.dtype], _p(dX), _p(X), rows, C, stream())


def tail_fwd(Y, s1, t1, pool, S, s2, t2, Out, amax, N, H, W, C):
    _lib.call("xcp_tail_fwd", DT[Y.dtype], _p(Y), _p(s1), _p(t1), 1 if pool else 0, _p(S), _p(s2), _p(t2), _p(Out),
              _p(amax), N, H, W, C, stream())


def maxpool_bwd(dOut, amax, dZ, N, H, W, C):
    _lib.call("xcp_maxpool_bwd", DT[dOut.dtype], _p(dOut), _p(amax), _p(dZ), N, H, W, C, stream())


def avgpool_fwd(Y, s, t, F, N, HW, C):
    _lib.call("xcp_avgpool_fwd", DT[Y.dtype], _p(Y), _p(s), _p(t), _p(F), N, HW, C, stream())


def avgpool_bwd(dF, Y, s, t, dZ, N, HW, C):
    _lib.call("xcp_avgpool_bwd", DT[Y.dtype], _p(dF), _p(Y), _p(s), _p(t), _p(dZ), N, HW, C, stream())


# ---------------------------------------------------------------- stem / packing
def conv1_fwd(X, W, Y, N, IH, IW):
    _lib.call("xcp_conv1_fwd", DT[Y.dtype], _p(X), _p(W), _p(Y), N, IH, IW, stream())


def conv1_wgrad(X, dY, out, N, IH, IW):
    R = _lib.call("xcp_conv1_wgrad_parts", N, IH, IW)
    part = torch.empty(R * 32 * 27, device=X.device, dtype=torch.float32)
    _lib.call("xcp_conv1_wgrad", DT[dY.dtype], _p(X), _p(dY), _p(part), N, IH, IW, stream())
    reduce_slabs(part, R, 32 * 27, out)


def permute3(inp, out, d0, d1, d2, perm):
    _lib.call("xcp_permute3", DT[out.dtype], _p(inp), _p(out), d0, d1, d2, perm[0], perm[1], perm[2], stream())


# ---------------------------------------------------------------- LSTM
def lstm_needs_whhT(H):
    return _lib.call("xcp_lstm_needs_whhT", H) != 0


def lstm_fwd(xproj, whh, whhT, bih, bhh, out, hprev, cst, gates, hn, cn, B, T, H):
    _lib.call("xcp_lstm_fwd", _p(xproj), _p(whh), _p(whhT), _p(bih), _p(bhh), _p(out), _p(hprev), _p(cst), _p(gates), _p(hn),
              _p(cn), B, T, H, stream())


def lstm_bwd(dout, dhn, dcn, whh, cst, gates, dgates, B, T, H):
    _lib.call("xcp_lstm_bwd", _p(dout), _p(dhn), _p(dcn), _p(whh), _p(cst), _p(gates), _p(dgates), B, T, H, stream())
