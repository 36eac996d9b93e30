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
    """The current HIP stream of the current device (callers enter ``device_guard`` first, so
    that is the device of the tensors the call works on)."""
    return torch.cuda.current_stream().cuda_stream


def device_guard(t):
    """Sets (and restores) the current device to ``t``'s for the duration of a block of launches:
    kernels are launched on the calling thread's current device and stream, and the reference
    calls these ops from the autograd engine's per-device threads and from
    nn.DataParallel.parallel_apply threads (train_audio.py:18, :38)."""
    return torch.cuda.device(t.device)


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


_op_log = None


def set_op_log(log):
    """Record every timed op's integer arguments and launch stream, in call order, into ``log``
    (a list; None turns it off): bench.py's XCP_BENCH_OP_ORDER dumps one step of it so that
    tools/prof_summary.py can put shapes on the launches of a rocprofv3 trace."""
    global _op_log
    _op_log = log


class _timed:
    def __init__(self, op, a):
        self.key = _timer.match(op, a) if _timer is not None else None
        if _op_log is not None:
            d = {k: v for k, v in a.items() if isinstance(v, int)}
            d["op"], d["stream"] = op, torch.cuda.current_stream().cuda_stream
            _op_log.append(d)

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
def gemm_nt(A, B, C, M, N, K, lda=None, ldb=None, ldc=None, stats=None, gather=(0, 0, 0, 0, 0, 1, 0), tile=0):
    """C[M,N] = A[M,K] B[N,K]^T (+ BN partial sums); tile 0 auto, 1 = 128x128, 2 = 256x256."""
    dt = DT[A.dtype]
    with _timed("gemm_nt", {"M": M, "N": N, "K": K, "stats": stats}):
        _lib.call("xcp_gemm_nt", dt, _p(A), lda or K, _p(B), ldb or K, _p(C), ldc or N, M, N, K, _p(stats), *gather,
                  tile, stream())


def gemm_tn(G, X, P, M, N, K, S, rows_per_split, ldg=None, ldx=None, gather=(0, 0, 0, 0, 0, 1, 0), tile=0):
    dt = DT[G.dtype]
    with _timed("gemm_tn", {"M": M, "N": N, "K": K, "ldg": ldg or N}):
        _lib.call("xcp_gemm_tn", dt, _p(G), ldg or N, _p(X), ldx or K, _p(P), M, N, K, S, rows_per_split, *gather,
                  tile, stream())


def nt_stat_rows(M):
    return _lib.call("xcp_gemm_nt_stat_rows", M)


def colreduce_f32(inp, S, L, out, G, accumulate=False, ld=None):
    _lib.call("xcp_colreduce_f32", _p(inp), S, L, ld or L, _p(out), G, 1 if accumulate else 0, stream())


def reduce_slabs(P, S, L, out, accumulate=False, ld=None):
    """out[L] (+)= sum_s P[s*ld : s*ld + L] (fp32, deterministic; two levels when S is large and
    L small).  ld (default L): slab stride, e.g. the padded channel pitch of depthwise partials."""
    g = _lib.call("xcp_colreduce_groups", S, L)
    if g:
        tmp = torch.empty(g * L, device=P.device, dtype=torch.float32)
        colreduce_f32(P, S, L, tmp, g, ld=ld)
        colreduce_f32(tmp, g, L, out, 1, accumulate)
    else:
        colreduce_f32(P, S, L, out, 1, accumulate, ld=ld)


class ReduceBatch:
    """Slab reductions collected and issued together (xcp_colreduce_multi, <= 16 jobs per launch):
    the engine batches one backbone block's weight-gradient reductions (pointwise split-K slabs,
    depthwise partials) into one or two launches instead of one or two per weight.  A job that
    reduce_slabs would split into two levels has its first level in the first launch and its
    second in the next; outputs are bitwise those of reduce_slabs."""

    def __init__(self):
        self.jobs = []

    def add(self, P, S, L, out, accumulate=False, ld=None):
        self.jobs.append((P, S, L, ld or L, out, bool(accumulate)))

    def flush(self):
        """enqueue every collected reduction on the current stream"""
        import ctypes
        if not self.jobs:
            return
        dev = self.jobs[0][0].device
        first, second = [], []
        for P, S, L, ld, out, acc in self.jobs:
            if L % 4 or ld % 4 or P.data_ptr() % 16 or out.data_ptr() % 16:
                reduce_slabs(P, S, L, out, acc, ld=ld)   # (float4 lanes only in the batched kernel)
                continue
            g = _lib.call("xcp_colreduce_groups", S, L)
            if g:
                tmp = torch.empty(g * L, device=dev, dtype=torch.float32)
                first.append((P, tmp, S, L, ld, g, 0))
                second.append((tmp, out, g, L, L, 1, int(acc)))
            else:
                first.append((P, out, S, L, ld, 1, int(acc)))
        for level in (first, second):
            for i in range(0, len(level), 16):
                chunk = level[i:i + 16]
                vals = [v for a, b, S, L, ld, G, acc in chunk for v in (a.data_ptr(), b.data_ptr(), S, L, ld, G, acc)]
                arr = (ctypes.c_longlong * len(vals))(*vals)
                _lib.call("xcp_colreduce_multi", ctypes.addressof(arr), len(chunk), stream())
        self.jobs = []


def weight_grad(G, X, M, N, K, out, gather=(0, 0, 0, 0, 0, 1, 0), ldg=None, ldx=None, tile=0, accumulate=False,
                batch=None):
    """out[N][K] (fp32) (+)= G[M][N]^T X[M][K].  batch (ReduceBatch): the slab reduction is added
    to it instead of launched here (the caller flushes it on this stream or one ordered after)."""
    rps = _lib.call("xcp_gemm_tn_rows_per_split", DT[G.dtype], gather[0], M, N, K, tile)
    S = (M + rps - 1) // rps
    P = torch.empty(S * N * K, device=G.device, dtype=torch.float32)
    gemm_tn(G, X, P, M, N, K, S, rps, ldg=ldg, ldx=ldx, gather=gather, tile=tile)
    if batch is not None:
        batch.add(P, S, N * K, out, accumulate)
    else:
        reduce_slabs(P, S, N * K, out, accumulate)


# ---------------------------------------------------------------- depthwise
def dw_fwd(act, X, Y, Wt, scale, shift, N, H, W, C):
    with _timed("dw_fwd", {"N": N, "H": H, "W": W, "C": C}):
        _lib.call("xcp_dw_fwd", DT[X.dtype], act, _p(X), _p(Y), _p(Wt), _p(scale), _p(shift), N, H, W, C, stream())


def sep_fwd_parts(dtype, N, H, W, cin, cout):
    """BN partial-sum rows of xcp_sep_fwd for this shape (0: not supported by the fused kernel)."""
    return _lib.call("xcp_sep_fwd_parts", DT[dtype], N, H, W, cin, cout)


def sep_fwd(act, X, scale, shift, dwt, pw, D, Y, part, N, H, W, cin, cout):
    """Fused depthwise 3x3 + pointwise 1x1 (+ BN partial sums of Y) of one entry-flow unit
    (csrc/sepfwd.hip): D = dw3x3(act(X)), Y = D pw^T, part [R][2][cout]."""
    check_gpu(X, D, Y)
    with _timed("sep_fwd", {"N": N, "H": H, "W": W, "C": cin, "CO": cout}):
        _lib.call("xcp_sep_fwd", DT[X.dtype], act, _p(X), _p(scale), _p(shift), _p(dwt), _p(pw), _p(D), _p(Y), _p(part),
                  N, H, W, cin, cout, stream())


def dw_bwd(act, dY, X, Wt, scale, shift, dX, dW_out, N, H, W, C, dRes=None, dSkip=None, skip_geom=(0, 0, 1),
           bn_stats=None, accumulate=False, Cw=None, skip_pre=False, reduce_stream=None, keep=None, batch=None,
           res_bn_input=None):
    """Returns (bnpart, P) -- the preceding BN's backward partial sums -- when bn_stats
    (that BN's Stats) is given, else (None, 0).  dW_out receives the weight gradient in the
    nn.Conv2d [C][1][3][3] order (accumulate: added to it); Cw (default C): channels of the
    weight when C is a padded channel pitch.  skip_pre: dSkip is a gradient of the same
    activation act(X) (it passes the activation mask and enters the BN partial sums).
    reduce_stream: run the weight-gradient slab reduction there (ordered after this launch);
    keep: a list that receives the scratch the reduce stream reads, for a caller that holds it
    until its stream has waited for the reduce stream (otherwise it is record_stream'ed);
    batch (ReduceBatch): the slab reduction is added to it instead (the caller flushes it after
    ordering its stream behind this launch, and keeps the scratch alive through ``keep``).
    res_bn_input (with dRes, no dSkip; bn_stats then the Stats of that BN): the partial sums are
    those of the BN whose output gradient is the final dX (after the residual add) and whose input
    is res_bn_input -- an identity-skip block boundary (xcp_dw_bwd_resbn)."""
    P = _lib.call("xcp_dw_bwd_chunks", N, H, W, C)
    part = torch.empty(P * C * 9, device=dY.device, dtype=torch.float32)
    bnpart = None
    if bn_stats is not None:
        bnpart = torch.empty(P * 2 * C, device=dY.device, dtype=torch.float32)
    if res_bn_input is not None:
        if dRes is None or dSkip is not None or bn_stats is None:
            raise ValueError("xcp.dw_bwd: res_bn_input needs dRes, no dSkip and the BN's bn_stats")
        _lib.call("xcp_dw_bwd_resbn", DT[dY.dtype], act, _p(dY), _p(X), _p(Wt), _p(scale), _p(shift), _p(dRes),
                  _p(dX), _p(part), _p(bnpart), _p(bn_stats["mean"]), _p(bn_stats["invstd"]), _p(res_bn_input),
                  N, H, W, C, stream())
    else:
        _lib.call("xcp_dw_bwd", DT[dY.dtype], act, _p(dY), _p(X), _p(Wt), _p(scale), _p(shift), _p(dRes), _p(dSkip),
                  skip_geom[0], skip_geom[1], skip_geom[2], int(skip_pre), _p(dX), _p(part), _p(bnpart),
                  _p(bn_stats["mean"]) if bn_stats is not None else 0,
                  _p(bn_stats["invstd"]) if bn_stats is not None else 0, N, H, W, C, stream())
    if batch is not None:
        batch.add(part, P, (Cw or C) * 9, dW_out, accumulate, ld=C * 9)
        if keep is not None:
            keep.append(part)
    elif reduce_stream is None:
        reduce_slabs(part, P, (Cw or C) * 9, dW_out, accumulate, ld=C * 9)
    else:
        reduce_stream.wait_stream(torch.cuda.current_stream(dY.device))
        with torch.cuda.stream(reduce_stream):
            reduce_slabs(part, P, (Cw or C) * 9, dW_out, accumulate, ld=C * 9)
        if keep is not None:
            keep.append(part)
        else:
            part.record_stream(reduce_stream)
            dW_out.record_stream(reduce_stream)
    return bnpart, (P if bnpart is not None else 0)


# ---------------------------------------------------------------- batchnorm


FIN_MAX_ROWS = 2048   # above this many partial rows, pre-reduce to FIN_GROUPS rows (fp64 sums, fp32 out)
FIN_GROUPS = 256


def _fold(part, R, CP):
    if R <= FIN_MAX_ROWS:
        return part, R
    G = min(FIN_GROUPS, R)   # (xcp_colreduce_f32 writes min(G, R) groups)
    p2 = torch.empty(G * 2 * CP, device=part.device, dtype=torch.float32)
    colreduce_f32(part, R, 2 * CP, p2, G)
    return p2, G


def finalize_stats(part, R, C, count, bn, train, out, CP=None):
    """part: fp32 [R][2][CP] partial sums -> out dict of mean/invstd/scale/shift (fp32 [CP], zero
    for the CP - C padding channels).  Updates bn running stats in place (train mode batch
    statistics)."""
    if not train:
        raise ValueError("finalize_stats computes batch statistics (train mode); use eval_stats")
    CP = CP or C
    track = bn["track"]
    part, R = _fold(part, R, CP)
    _lib.call("xcp_bn_finalize_part", _p(part), R, C, CP, float(count), _p(bn["weight"]), _p(bn["bias"]),
              _p(bn["running_mean"]) if track else 0, _p(bn["running_var"]) if track else 0, float(bn["momentum"]),
              float(bn["eps"]), _p(out["mean"]), _p(out["invstd"]), _p(out["scale"]), _p(out["shift"]), stream())


def _bn_finalize(p2, G, C, count, bn, train, out, CP=None):
    mom = bn["momentum"]
    _lib.call("xcp_bn_finalize", _p(p2), G, C, CP or C, float(count), _p(bn["weight"]), _p(bn["bias"]),
              _p(bn["running_mean"]) if (train and bn["track"]) or not train else 0,
              _p(bn["running_var"]) if (train and bn["track"]) or not train else 0, float(mom), float(bn["eps"]),
              1 if train else 0, _p(out["mean"]), _p(out["invstd"]), _p(out["scale"]), _p(out["shift"]), stream())


def eval_stats(C, bn, out, device, CP=None):
    p2 = torch.zeros(2 * (CP or C), device=device, dtype=torch.float64)
    _bn_finalize(p2, 1, C, 1.0, bn, False, out, CP)


def row_stats(X, rows, C):
    R = _lib.call("xcp_chanred_parts", rows, C)
    part = torch.empty(R * 2 * C, device=X.device, dtype=torch.float32)
    _lib.call("xcp_row_stats", DT[X.dtype], _p(X), rows, C, _p(part), stream())
    return part, R


def bn_backward_coef(dZ, Y, rows, C, bn, st, dgamma, dbeta, part=None, R=0, relu=False, accumulate=False, CP=None,
                     narrow=False):
    """BatchNorm2d backward (train-mode batch stats) up to the per-channel coefficients:
    returns coef fp32 [3][C] (alpha, bcoef, delta: dY = alpha*dZ' + bcoef*Y + delta, dZ' the
    ReLU-masked dZ when relu) and writes (accumulate: adds to) dgamma/dbeta.
    ``part`` ([R][2][CP] partial (sum dz, sum dz*zhat)) may come fused from the
    producer of dZ; otherwise it is reduced here.  relu=True: dZ is the gradient of
    relu(bn(Y)) (the ReLU mask is recomputed from Y and st's scale/shift).  CP (default C):
    channel pitch of dZ / Y; coef then has CP entries per coefficient, zero for the padding.  narrow: the
    finalize in 4-wave workgroups (room beside a kernel holding every CU; XCP_FIN_NARROW)."""
    CP = CP or C
    ms, mt = (_p(st["scale"]), _p(st["shift"])) if relu else (0, 0)
    dev, dt = Y.device, Y.dtype
    if part is None:
        R = _lib.call("xcp_chanred_parts", rows, CP)
        part = torch.empty(R * 2 * CP, device=dev, dtype=torch.float32)
        _lib.call("xcp_bn_bwd_reduce", DT[dt], _p(dZ), _p(Y), _p(st["mean"]), _p(st["invstd"]), ms, mt, rows, CP,
                  _p(part), stream())
    elif relu:
        raise ValueError("a fused partial cannot carry the ReLU mask")
    coef = torch.empty(3 * CP, device=dev, dtype=torch.float32)
    part, R = _fold(part, R, CP)
    _lib.call("xcp_bn_bwd_finalize_part", _p(part), R, C, CP, float(rows), _p(bn["weight"]), _p(st["mean"]),
              _p(st["invstd"]), _p(coef), _p(coef[CP:]), _p(coef[2 * CP:]), _p(dgamma), _p(dbeta),
              (1 if accumulate else 0) | (2 if narrow else 0), stream())
    return coef


def bn_backward(dZ, Y, rows, C, bn, st, dY, dgamma, dbeta, part=None, R=0, relu=False, accumulate=False):
    """dY = BatchNorm2d backward (train-mode batch stats) of dZ; writes (accumulate: adds to)
    dgamma/dbeta (see bn_backward_coef)."""
    coef = bn_backward_coef(dZ, Y, rows, C, bn, st, dgamma, dbeta, part=part, R=R, relu=relu, accumulate=accumulate)
    bn_apply_coef(dZ, Y, dY, coef, st, rows, C, relu)


def bn_apply_coef(dZ, Y, dY, coef, st, rows, C, relu=False):
    """dY = alpha*dZ' + bcoef*Y + delta (coef from bn_backward_coef; dZ' ReLU-masked when relu);
    C: the channel pitch (coef has C entries per coefficient)"""
    ms, mt = (_p(st["scale"]), _p(st["shift"])) if relu else (0, 0)
    _lib.call("xcp_bn_bwd_apply", DT[Y.dtype], _p(dZ), _p(Y), _p(dY), _p(coef), _p(coef[C:]), _p(coef[2 * C:]), ms,
              mt, rows, C, stream())


def unit_bwd_rows_per_split(dtype, M, CO, CI):
    """rows per split of the fused pointwise + BN unit backward (0: shape not supported)"""
    return _lib.call("xcp_unit_bwd_rows_per_split", DT[dtype], M, CO, CI)


def unit_bwd(G, Y, coef, Wt, X, dD, M, CO, CI, dW_out, accumulate=False):
    """Fused unit backward: dY = alpha*G + bcoef*Y + delta (coef from bn_backward_coef, never
    stored), dD[M][CI] = dY Wt^T (Wt: [CI][CO]), dW_out[CO][CI] (+)= dY^T X."""
    rps = unit_bwd_rows_per_split(G.dtype, M, CO, CI)
    if rps <= 0:
        raise ValueError(f"xcp.unit_bwd: unsupported shape M={M} CO={CO} CI={CI} dtype={G.dtype}")
    S = (M + rps - 1) // rps
    P = torch.empty(S * CO * CI, device=G.device, dtype=torch.float32)
    with _timed("unit_bwd", {"M": M, "CO": CO, "CI": CI}):
        _lib.call("xcp_unit_bwd", DT[G.dtype], _p(G), _p(Y), _p(coef), _p(coef[CO:]), _p(coef[2 * CO:]), _p(Wt),
                  _p(X), _p(dD), _p(P), M, CO, CI, S, rps, stream())
    reduce_slabs(P, S, CO * CI, dW_out, accumulate)


def bn_act(X, Y, scale, shift, relu, rows, C):
    _lib.call("xcp_bn_act", DT[X.dtype], _p(X), _p(Y), _p(scale), _p(shift), 1 if relu else 0, rows, C, stream())


def bn_act_strided(X, Y, scale, shift, relu, N, H, W, OH, OW, S, C):
    """Y[n,oh,ow] = act(X[n, oh*S, ow*S] * scale + shift) (NHWC pixel rows of C channels)."""
    _lib.call("xcp_bn_act_strided", DT[X.dtype], _p(X), _p(Y), _p(scale), _p(shift), int(relu), N, H, W, OH, OW, S, C,
              stream())


def relu_bwd(dX, X, rows, C):
    _lib.call("xcp_relu_bwd", DT[dX.dtype], _p(dX), _p(X), rows, C, stream())


def tail_fwd(Y, s1, t1, pool, S, s2, t2, Out, amax, N, H, W, C):
    _lib.call("xcp_tail_fwd", DT[Y.dtype], _p(Y), _p(s1), _p(t1), 1 if pool else 0, _p(S), _p(s2), _p(t2), _p(Out),
              _p(amax), N, H, W, C, stream())


def maxpool_bwd(dOut, amax, dZ, N, H, W, C):
    _lib.call("xcp_maxpool_bwd", DT[dOut.dtype], _p(dOut), _p(amax), _p(dZ), N, H, W, C, stream())


def maxpool_bwd_bnred(dOut, amax, dZ, Y, st, N, H, W, C):
    """maxpool_bwd into dZ plus the BN-backward reduce of dZ against Y (st: that BN's Stats)
    in one pass.  Returns (part [P][2][C], P) for bn_backward(part=...)."""
    R = _lib.call("xcp_maxpool_bwd_bnred_parts", N, H, W, C)
    part = torch.empty(R * 2 * C, device=Y.device, dtype=torch.float32)
    _lib.call("xcp_maxpool_bwd_bnred", DT[dOut.dtype], _p(dOut), _p(amax), _p(dZ), _p(Y), _p(st["mean"]),
              _p(st["invstd"]), N, H, W, C, _p(part), stream())
    return part, R


def avgpool_fwd(Y, s, t, F, N, HW, C):
    _lib.call("xcp_avgpool_fwd", DT[Y.dtype], _p(Y), _p(s), _p(t), _p(F), N, HW, C, stream())


def avgpool_bwd(dF, Y, s, t, dZ, N, HW, C):
    _lib.call("xcp_avgpool_bwd", DT[Y.dtype], _p(dF), _p(Y), _p(s), _p(t), _p(dZ), N, HW, C, stream())


# ---------------------------------------------------------------- stem / packing
def conv1_fwd(X, W, Y, N, IH, IW):
    _lib.call("xcp_conv1_fwd", DT[Y.dtype], _p(X), _p(W), _p(Y), N, IH, IW, stream())


def conv1_fwd_stats(X, W, Y, N, IH, IW):
    """conv1 forward + BN1 partial sums of the stored output: returns (part [R][2][32], R)"""
    R = _lib.call("xcp_conv1_fwd_parts", N, IH, IW)
    part = torch.empty(R * 2 * 32, device=X.device, dtype=torch.float32)
    _lib.call("xcp_conv1_fwd_stats", DT[Y.dtype], _p(X), _p(W), _p(Y), _p(part), N, IH, IW, stream())
    return part, R


def conv1_wgrad(X, dY, out, N, IH, IW, accumulate=False):
    R = _lib.call("xcp_conv1_wgrad_parts", N, IH, IW)
    part = torch.empty(R * 32 * 27, device=X.device, dtype=torch.float32)
    _lib.call("xcp_conv1_wgrad", DT[dY.dtype], _p(X), _p(dY), _p(part), N, IH, IW, stream())
    reduce_slabs(part, R, 32 * 27, out, accumulate)


def conv1_wgrad_fused(dtype, IH, IW):
    """True when conv1_wgrad_bn takes the shape"""
    return _lib.call("xcp_conv1_wgrad_fused", DT[dtype], IH, IW) == 1


def conv1_wgrad_bn(X, dZ, Y, coef, st, out, N, IH, IW, C, relu=True, accumulate=False):
    """conv1's weight gradient with BN1's backward apply fused: as bn_apply_coef(dZ, Y, dC1, coef, st, ...,
    relu) followed by conv1_wgrad(X, dC1, out, ...), without storing dC1 (C: the channel pitch of coef)."""
    R = _lib.call("xcp_conv1_wgrad_parts", N, IH, IW)
    part = torch.empty(R * 32 * 27, device=X.device, dtype=torch.float32)
    ms, mt = (_p(st["scale"]), _p(st["shift"])) if relu else (0, 0)
    with _timed("conv1_wgrad_bn", {"N": N, "IH": IH, "IW": IW}):
        _lib.call("xcp_conv1_wgrad_bn", DT[dZ.dtype], _p(X), _p(dZ), _p(Y), _p(coef), _p(coef[C:]), _p(coef[2 * C:]),
                  ms, mt, _p(part), N, IH, IW, stream())
    reduce_slabs(part, R, 32 * 27, out, accumulate)


def frames_u8_to_f32(frames, lengths, out):
    """frames: uint8 [B, Tmax, H, W, 3] (device), lengths: int32 [B] (device) -> out fp32
    [B, Tmax, 3, H, W] = frames / 255, zero past each clip's length (video_dataloader.py:35, :59-64)."""
    check_gpu(frames, lengths, out)
    B, T, H, W, C = frames.shape
    if C != 3 or frames.dtype != torch.uint8 or lengths.dtype != torch.int32 or out.dtype != torch.float32 \
            or tuple(out.shape) != (B, T, 3, H, W) or not (frames.is_contiguous() and out.is_contiguous()):
        raise ValueError("frames_u8_to_f32: expects uint8 [B,T,H,W,3], int32 [B] and fp32 [B,T,3,H,W]")
    _lib.call("xcp_frames_u8_to_f32", _p(frames), _p(lengths), _p(out), B, T, H, W, stream())


def frames_prep(frames, lengths, size=None, dtype=torch.float32, channels_last=False):
    """uint8 [B, T, H, W, 3] frames (device) + int32 [B] lengths -> the clip tensor
    [B, T, 3, OH, OW] of ``dtype`` = F.interpolate(frames / 255, size, bilinear,
    align_corners=False) (no resize when size is None or (H, W)); zero past each clip's length.
    channels_last: the storage is [B, T, OH, OW, 3] (the returned tensor is its permuted view)."""
    check_gpu(frames, lengths)
    B, T, H, W, C = frames.shape
    if C != 3 or frames.dtype != torch.uint8 or lengths.dtype != torch.int32 or dtype not in DT:
        raise ValueError("frames_prep: expects uint8 [B,T,H,W,3], int32 [B], fp32 / bf16 output")
    OH, OW = (H, W) if size is None else size
    frames = frames.contiguous()
    if channels_last:
        out = torch.empty((B, T, OH, OW, 3), device=frames.device, dtype=dtype)
    else:
        out = torch.empty((B, T, 3, OH, OW), device=frames.device, dtype=dtype)
    _lib.call("xcp_frames_prep", _p(frames), _p(lengths), _p(out), B, T, H, W, OH, OW, DT[dtype],
              1 if channels_last else 0, stream())
    return out.permute(0, 1, 4, 2, 3) if channels_last else out


def resize_bilinear(x, size):
    """F.interpolate(x, size, mode="bilinear", align_corners=False) for fp32 NCHW x on the GPU
    (the XceptionLSTMA front end, XceptionLSTMA.py:46)."""
    check_gpu(x)
    if x.dtype != torch.float32 or x.dim() != 4:
        raise ValueError("resize_bilinear: expects fp32 [N, C, H, W]")
    x = x.contiguous()
    N, C, IH, IW = x.shape
    OH, OW = size
    out = torch.empty((N, C, OH, OW), device=x.device, dtype=torch.float32)
    _lib.call("xcp_resize_bilinear", _p(x), _p(out), N * C, IH, IW, OH, OW, stream())
    return out


def conv3x3_parts(mode, N, IH, IW):
    return _lib.call("xcp_conv3x3_parts", mode, N, IH, IW)


def conv3x3(mode, X, W, Y, stats, N, IH, IW, in_scale=None, in_shift=None):
    """Stem conv2 as a direct MFMA conv (bf16): mode 0 forward 32->64 (+ BN partial sums),
    mode 1 its input gradient 64->32 (W = the [32][9][64] transposed kernel).  in_scale /
    in_shift (mode 0): X is conv1's raw output, BN1 + ReLU applied on load."""
    if X.dtype != torch.bfloat16:
        raise ValueError("xcp_conv3x3 is bf16 only")
    _lib.call("xcp_conv3x3", mode, _p(X), _p(W), _p(Y), _p(stats), N, IH, IW, _p(in_scale), _p(in_shift), stream())


def conv3x3_wgrad_parts(N, IH, IW):
    return _lib.call("xcp_conv3x3_wgrad_parts", N, IH, IW)


def conv3x3_wgrad(dY, X, out, N, IH, IW, in_scale=None, in_shift=None):
    """out[64][9*32] fp32 = weight gradient of the stem conv2 (tap-major, [co][kh*3+kw][ci])
    from dY [N,IH-2,IW-2,64] and X [N,IH,IW,32] (bf16): per-workgroup slabs + colreduce.
    in_scale / in_shift: X is conv1's raw output, BN1 + ReLU applied on load."""
    if dY.dtype != torch.bfloat16 or X.dtype != torch.bfloat16:
        raise ValueError("xcp_conv3x3_wgrad is bf16 only")
    S = conv3x3_wgrad_parts(N, IH, IW)
    if S <= 0:
        raise ValueError("xcp_conv3x3_wgrad: unsupported width")
    P = torch.empty(S * 64 * 288, device=dY.device, dtype=torch.float32)
    _lib.call("xcp_conv3x3_wgrad", _p(dY), _p(X), _p(P), N, IH, IW, _p(in_scale), _p(in_shift), stream())
    reduce_slabs(P, S, 64 * 288, out)


def permute3(inp, out, d0, d1, d2, perm):
    _lib.call("xcp_permute3", DT[out.dtype], _p(inp), _p(out), d0, d1, d2, perm[0], perm[1], perm[2], stream())


class PermuteBatch:
    """A fixed list of permute3 jobs (fp32 source -> packed destination) run as one launch.
    The device job table is rebuilt only when a source or destination pointer changes."""

    def __init__(self):
        self._key = None
        self._table = None
        self._nblocks = 0

    def run(self, jobs):
        """jobs: list of (src fp32 tensor, dst tensor, d0, d1, d2, perm[, s0]): output element
        (o0, o1, o2) of the permuted [od0][od1][od2] array goes to dst[o0*s0 + o1*od2 + o2]
        (s0 default od1*od2; larger for a padded destination, whose padding is left alone)."""
        jobs = [j if len(j) == 7 else (*j, None) for j in jobs]
        key = tuple((s.data_ptr(), d.data_ptr(), d0, d1, d2, tuple(pm), d.dtype, s0)
                    for s, d, d0, d1, d2, pm, s0 in jobs)
        if key != self._key:
            rows, blk = [], 0
            for s, d, d0, d1, d2, pm, s0 in jobs:
                n = d0 * d1 * d2
                dims = (d0, d1, d2)
                od0, od1, od2 = dims[pm[0]], dims[pm[1]], dims[pm[2]]
                s1 = od2
                s0 = s0 or od1 * od2
                if sorted(pm) != [0, 1, 2] or s.numel() != n or s0 < od1 * od2 or d.numel() < (od0 - 1) * s0 + od1 * od2 \
                        or s.dtype != torch.float32 or not s.is_contiguous() or not d.is_contiguous():
                    raise ValueError("permute job: bad permutation, size, dtype or layout")
                check_gpu(s, d)
                rows.append([s.data_ptr(), d.data_ptr(), d0, d1, d2, pm[0], pm[1], pm[2], DT[d.dtype], blk, s0, s1])
                blk += _lib.call("xcp_permute3_blocks", d0, d1, d2, pm[0], pm[1], pm[2], s0, s1)
            self._table = torch.tensor(rows, dtype=torch.int64).to(jobs[0][1].device)
            self._nblocks, self._key = blk, key
        _lib.call("xcp_permute3_batch", _p(self._table), len(jobs), self._nblocks, stream())


# ---------------------------------------------------------------- diagnostics
def clock_probe(device, launches=8, iters=40000):
    """Shader clock (MHz) the chip holds under a bf16 MFMA load: ``launches`` back-to-back
    probe launches (one workgroup per CU, ~0.6 ms each), median over the last launch's
    workgroups of cycles / real-time ticks x 100 MHz (MI355X_MICROARCH.md, DVFS item 6)."""
    blocks = torch.cuda.get_device_properties(device).multi_processor_count
    out = torch.zeros(2 * blocks + 256, device=device, dtype=torch.int64)
    with torch.cuda.device(device):
        for _ in range(launches):
            _lib.call("xcp_clock_probe", out.data_ptr(), blocks, iters, stream())
        v = out[:2 * blocks].view(blocks, 2).cpu()
    mhz = (v[:, 0].double() / v[:, 1].double().clamp(min=1)) * 100.0
    return float(mhz.median())


# ---------------------------------------------------------------- LSTM
# kernel: 0 = automatic (register-resident for H 64 / 128, per-step kernels for H 256-1024),
# 1 = the generic kernels (tests pin them at shapes the specialised kernels also cover)
def lstm_needs_whhT(B, H, kernel=0):
    return _lib.call("xcp_lstm_needs_whhT", B, H, kernel) != 0


def lstm_fwd(xproj, whh, whhT, bih, bhh, out, hprev, cst, gates, hn, cn, B, T, H, kernel=0):
    _lib.call("xcp_lstm_fwd", _p(xproj), _p(whh), _p(whhT), _p(bih), _p(bhh), _p(out), _p(hprev), _p(cst), _p(gates), _p(hn),
              _p(cn), B, T, H, kernel, stream())


def lstm_sync_error():
    """1 if a persistent LSTM launch gave up waiting for its workgroups since the last call (its
    outputs are invalid then), else 0; synchronises the device and clears the flags."""
    return _lib.call("xcp_lstm_sync_error")


def lstm_bwd(dout, dhn, dcn, whh, cst, gates, dgates, B, T, H, kernel=0):
    # per-step kernels: cell-gradient carry [B][H] + W_hh^T [H][4H]; persistent kernels: the dh partials
    # [2][B][H / 4][H / 4][4] (include/xcp.h)
    work = torch.empty(max(B * H + 4 * H * H, B * H * H // 2), device=whh.device, dtype=torch.float32)
    _lib.call("xcp_lstm_bwd", _p(dout), _p(dhn), _p(dcn), _p(whh), _p(cst), _p(gates), _p(dgates), _p(work), B, T, H,
              kernel, stream())

