"""Whole-backbone executor for Xception (forward + backward) on the xcp kernels.

The reference runs ``Xception.forward`` (Xception.py:167-201) module by module
through ATen; here one engine walks the same graph with the hand-written gfx950
kernels of ``libxcp.so`` and keeps activations NHWC in HBM:

* BatchNorm is never materialised inside a block: the pointwise GEMM epilogue
  emits the batch statistics, and BN-apply + ReLU is folded into the load of the
  next depthwise conv (``ACT_BNRELU``); only block outputs (``x += skip``,
  Xception.py:98) and the stem output are written.
* Backward reuses the saved raw tensors: the fused depthwise backward recomputes
  the BN+ReLU input on the fly, applies the ReLU mask and adds the identity /
  strided skip gradients.

One engine serves one ``Xception`` module; it is driven through
``XceptionFunction`` so autograd sees a single node whose inputs are the frames and
every backbone parameter.

Gradient delivery has two modes:

* default: the backward returns one fp32 gradient per parameter to autograd, which
  accumulates it into ``param.grad`` (tensor hooks, post-accumulate-grad hooks,
  ``torch.autograd.grad`` and ``backward(inputs=...)`` all behave as for any module);
* gradient sink (``xcp.ddp.GradBuckets(..., module=model)`` registers one): the kernels
  accumulate straight into the ``param.grad`` views of the sink's flat buffer and the
  sink is told after each block which parameters are final, so it all-reduces a bucket
  while the earlier blocks' backward is still running.
"""
import contextlib
import os
import math

import torch
import torch.nn as nn

from . import ops
from .ops import ACT_BNRELU, ACT_NONE, ACT_RELU


def _bn_ref(m):
    return {"weight": m.weight, "bias": m.bias, "running_mean": m.running_mean, "running_var": m.running_var,
            "eps": m.eps, "momentum": m.momentum, "track": m.track_running_stats, "module": m}


class _Unit:
    """relu? -> SeparableConv2d -> BatchNorm2d, one element of Block.rep (Xception.py:61-79)."""

    def __init__(self, sep, bn, relu, name, bn_name):
        self.sep, self.bn, self.relu, self.name, self.bn_name = sep, bn, relu, name, bn_name
        self.cin = sep.conv1.in_channels
        self.cout = sep.pointwise.out_channels
        if sep.conv1.kernel_size != (3, 3) or sep.conv1.stride != (1, 1) or sep.conv1.padding != (1, 1):
            raise NotImplementedError("xcp engine supports the Xception 3x3/s1/p1 separable convs only")
        if sep.conv1.bias is not None or sep.pointwise.bias is not None:
            raise NotImplementedError("xcp engine: separable convs are bias-free in Xception")


class _Block:
    def __init__(self, blk, name):
        self.name = name
        self.units = []
        self.pool = False
        mods = list(blk.rep)
        i, relu = 0, False
        while i < len(mods):
            m = mods[i]
            if isinstance(m, nn.ReLU):
                relu = True
                i += 1
            elif m.__class__.__name__ == "SeparableConv2d":
                bn = mods[i + 1]
                assert isinstance(bn, nn.BatchNorm2d)
                self.units.append(_Unit(m, bn, relu, f"{name}.rep.{i}", f"{name}.rep.{i + 1}"))
                relu = False
                i += 2
            elif isinstance(m, nn.MaxPool2d):
                if (m.kernel_size, m.stride, m.padding) not in ((3, 2, 1), ((3, 3), (2, 2), (1, 1))):
                    raise NotImplementedError("xcp engine: MaxPool2d(3, 2, 1) only")
                self.pool = True
                i += 1
            else:
                raise NotImplementedError(f"xcp engine: unexpected module {type(m)} in {name}.rep")
        for u in self.units[1:]:
            if not u.relu:
                raise NotImplementedError("xcp engine: inner separable convs must be preceded by ReLU")
        self.skip = blk.skip
        self.skipbn = getattr(blk, "skipbn", None) if blk.skip is not None else None
        self.stride = blk.skip.stride[0] if blk.skip is not None else 1
        if self.pool and self.skip is None:
            raise NotImplementedError("xcp engine: a pooled block needs a conv skip")
        if self.skip is not None and self.stride != (2 if self.pool else 1):
            raise NotImplementedError("xcp engine: skip stride must match the pooling")
        self.cin = self.units[0].cin
        self.cout = self.units[-1].cout


class Stats:
    __slots__ = ("mean", "invstd", "scale", "shift")

    def __init__(self, C, dev):
        buf = torch.empty(4 * C, device=dev, dtype=torch.float32)
        self.mean, self.invstd, self.scale, self.shift = buf[:C], buf[C:2 * C], buf[2 * C:3 * C], buf[3 * C:]

    def __getitem__(self, k):
        return getattr(self, k)


# pointwise weight gradients on a side stream (XCP_WGRAD_STREAM=0 keeps them in order)
WGRAD_SIDE_STREAM = os.environ.get("XCP_WGRAD_STREAM", "1") != "0"
# fused BN-apply + pointwise dgrad + wgrad for the narrow units (csrc/unitbwd.hip);
# XCP_FUSED_UNIT_BWD=0 runs the three-kernel sequence (A/B and parity cross-checks)
FUSED_UNIT_BWD = os.environ.get("XCP_FUSED_UNIT_BWD", "1") != "0"
# XCP_STEM_FUSED=0 materialises relu(bn2(conv2)) at full resolution for block1 (A/B and parity
# cross-checks); by default block1's first depthwise conv applies BN2 + ReLU on load
STEM_FUSED = os.environ.get("XCP_STEM_FUSED", "1") != "0"
# an identity-skip block boundary's BN partial sums from the next block's first depthwise backward
# (xcp_dw_bwd_resbn) instead of a per-channel reduce pass (XCP_RESBN=1; default off until measured)
RESBN = os.environ.get("XCP_RESBN", "0") == "1"
STEM_WGRAD_SIDE = WGRAD_SIDE_STREAM and os.environ.get("XCP_STEM_WGRAD_SIDE", "1") != "0"
SIDE_PRIO_LOW = os.environ.get("XCP_SIDE_PRIO", "") == "low"
# BN1's backward coefficients before the side-stream conv2 weight gradient is launched
# (XCP_STEM_BN1_FIRST=0: after it, the round-2 order; A/B)
STEM_BN1_FIRST = os.environ.get("XCP_STEM_BN1_FIRST", "1") != "0"
# conv1's weight gradient forms BN1's backward apply (+ ReLU mask) on load instead of reading a stored
# dC1 (xcp_conv1_wgrad_bn; XCP_CONV1_BN_FUSED=0: bn_bwd_apply + conv1_wgrad, A/B)
CONV1_BN_FUSED = os.environ.get("XCP_CONV1_BN_FUSED", "1") != "0"
# conv2's weight gradient launched on the weight-gradient stream before conv2's input gradient, so it runs
# beside the dgrad, BN1's coefficients and conv1's weight gradient instead of after them and the backward
# no longer ends waiting for it (+0.2-0.5 % in two interleaved rounds, profiles/r04_stem_order_ab.txt;
# XCP_STEM_WGRAD_EARLY=0: after BN1's coefficients)
STEM_WGRAD_EARLY = os.environ.get("XCP_STEM_WGRAD_EARLY", "1") != "0"
# BN1's backward finalize in 4-wave workgroups (XCP_FIN_NARROW) while conv2's weight gradient holds every CU on the
# side stream: the 16-wave workgroup found no SIMD with room for 4 of its waves and waited for the whole weight
# gradient (144 us per step, profiles/r06_conv3_wgrad_ab.txt).  XCP_STEM_FIN_NARROW=0: the 16-wave form (A/B)
STEM_FIN_NARROW = os.environ.get("XCP_STEM_FIN_NARROW", "1") != "0"
# BN1's batch statistics from conv1's forward (xcp_conv1_fwd_stats; XCP_CONV1_STATS_FUSED=0: a per-channel
# reduce over the stored output, A/B)
CONV1_STATS_FUSED = os.environ.get("XCP_CONV1_STATS_FUSED", "1") != "0"
# depthwise weight-gradient slab reductions on the weight-gradient stream (XCP_DW_REDUCE_SIDE=0:
# on the main stream right after each depthwise backward)
DW_REDUCE_SIDE = WGRAD_SIDE_STREAM and os.environ.get("XCP_DW_REDUCE_SIDE", "1") != "0"
# one block's weight-gradient slab reductions batched into one or two launches (XCP_REDUCE_BATCH=0:
# one launch per weight, as they are produced)
REDUCE_BATCH = os.environ.get("XCP_REDUCE_BATCH", "1") != "0"
# XCP_NT_ONESHOT=1: the big pointwise GEMMs on the one-shot 256x256 kernel instead of its
# persistent form (gemm.hip tile 4 vs 0; A/B); XCP_NT_TILE=<t> pins any gemm.hip tile choice for them
# block1's units (147^2, 64 -> 128 and 128 -> 128) run depthwise + pointwise + BN sums as one kernel
# (csrc/sepfwd.hip): the depthwise output goes to the MFMAs through LDS instead of back through HBM
# (XCP_SEP_FUSED=0: the two kernels; A/B)
SEP_FUSED = os.environ.get("XCP_SEP_FUSED", "1") != "0"
# ... from these frame widths on: the kernel computes whole 80-pixel half rows (two for 128 outputs, one
# for 256) with four barriers each, so on narrow frames most of its work is padding and the per-row
# barriers dominate (64^2 clips, block1 at 29^2: 848 us per launch against the two kernels' ~300, C4
# line 1847 -> 2279 clips/s with the two kernels, profiles/r06_c4_ab.txt).  XCP_SEP_NARROW=1: every
# width the kernel supports (A/B)
SEP_MIN_W = {128: 0, 256: 0} if os.environ.get("XCP_SEP_NARROW", "0") == "1" else {128: 120, 256: 64}
# the stem conv2 (forward and weight gradient) applies BN1 + ReLU on load instead of reading a
# materialised relu(bn1(conv1)) (XCP_CONV2_ACTIN=0: bn_act + the plain conv; A/B)
CONV2_ACT_ON_LOAD = os.environ.get("XCP_CONV2_ACTIN", "1") != "0"
# XCP_WGRAD_FIRST=1: a unit's pointwise weight gradient launched on the side stream before its input
# gradient, so the two overlap (A/B; +0.40 % on one box, -0.17 % on another: profiles/r05_wgrad_first_ab.txt;
# off: the side stream waits for the input gradient)
WGRAD_FIRST = os.environ.get("XCP_WGRAD_FIRST", "0") == "1"
# XCP_WGRAD_DEFER=1: a unit's pointwise weight gradient is launched on the side stream after the NEXT unit's
# input gradient instead of its own, so it runs beside the memory-bound depthwise backward / BN apply that
# follow rather than beside the next input-gradient GEMM (A/B)
WGRAD_DEFER = os.environ.get("XCP_WGRAD_DEFER", "0") == "1"
# XCP_SKIP_WGRAD_LATE=1: a block's skip-conv weight gradient launched on the side stream after the block's
# units instead of before them (A/B: off keeps it beside the block's own depthwise backward)
SKIP_WGRAD_LATE = os.environ.get("XCP_SKIP_WGRAD_LATE", "0") == "1"
NT_TILE = int(os.environ.get("XCP_NT_TILE", "4" if os.environ.get("XCP_NT_ONESHOT", "0") == "1" else "0"))
# Channel pitch of the 728-channel flow (block3 .. block12): 736, so every pixel row starts on a
# 64-B (bf16) / 128-B (fp32) boundary.  The 8 padding channels are zero throughout: zero rows /
# columns in the packed weights, zero BN scale / shift / backward coefficients.  XCP_PAD_728=0
# keeps the dense 728 pitch, XCP_PAD_728=<pitch> (a multiple of 8 above 728) sets another (A/B).
_pad = os.environ.get("XCP_PAD_728", "736")
PAD_PITCH = {} if _pad == "0" else {728: int(_pad)}
if PAD_PITCH and (PAD_PITCH[728] < 728 or PAD_PITCH[728] % 8):
    raise ValueError("XCP_PAD_728 must be 0 or a multiple of 8 >= 728")


def pc(c):
    """channel pitch of a c-channel activation"""
    return PAD_PITCH.get(c, c)


class XceptionEngine:
    def __init__(self, model, dtype=torch.bfloat16):
        if dtype not in (torch.float32, torch.bfloat16):
            raise ValueError("xcp engine dtype must be float32 (parity) or bfloat16")
        self.model = model
        self.dtype = dtype
        self.blocks = [_Block(getattr(model, f"block{i}"), f"block{i}") for i in range(1, 13)]
        self.exit_units = [_Unit(model.conv3, model.bn3, False, "conv3", "bn3"),
                           _Unit(model.conv4, model.bn4, True, "conv4", "bn4")]
        c1, c2 = model.conv1, model.conv2
        if (c1.in_channels, c1.out_channels, c1.kernel_size, c1.stride, c1.padding) != (3, 32, (3, 3), (2, 2), (0, 0)):
            raise NotImplementedError("xcp engine: Xception stem conv1 must be 3->32 3x3 s2 p0")
        if (c2.in_channels, c2.out_channels, c2.kernel_size, c2.stride, c2.padding) != (32, 64, (3, 3), (1, 1), (0, 0)):
            raise NotImplementedError("xcp engine: Xception stem conv2 must be 32->64 3x3 s1 p0")
        self.bn_modules = [m for m in model.modules() if isinstance(m, nn.BatchNorm2d)]
        self._pack_key = None
        self._packed = {}
        self._packed_bwd_key = None
        self._bufs = {}
        self._pack_fwd, self._pack_bwd = ops.PermuteBatch(), ops.PermuteBatch()

    @property
    def grad_sink(self):
        """The gradient sink registered on the module (xcp.ddp.GradBuckets(module=...)), or None."""
        return getattr(self.model, "_xcp_grad_sink", None)

    def _side_stream(self, dev):
        st = getattr(self, "_side", None)
        if st is None or st.device != dev:
            # XCP_SIDE_PRIO=low: the weight-gradient stream at the least priority the device offers
            # (below the default stream's when the range has one), so the dispatcher prefers the
            # main stream's workgroups (A/B; the default creates it at the default priority)
            prio = torch.cuda.Stream.priority_range()[0] if SIDE_PRIO_LOW else 0
            st = self._side = torch.cuda.Stream(dev, priority=prio)
        return st

    # ------------------------------------------------------------ parameters
    def named_params(self):
        """Backbone parameters in a fixed order (the autograd inputs).  On an nn.DataParallel
        replica the parameters are the broadcast copies DataParallel set as plain attributes
        (``_former_parameters``, same names and order): gradients w.r.t. them flow back to the
        original parameters through DataParallel's broadcast."""
        if getattr(self.model, "_is_replica", False):
            out = []
            for mn, mod in self.model.named_modules():
                for k, t in getattr(mod, "_former_parameters", {}).items():
                    n = f"{mn}.{k}" if mn else k
                    if t is not None and not n.startswith("fc."):
                        out.append((n, t))
            return out
        return [(n, p) for n, p in self.model.named_parameters() if not n.startswith("fc.")]

    def _version_key(self):
        return tuple((p.data_ptr(), p._version) for _, p in self.named_params()) + (self.dtype,)

    def _buf(self, name, n, dtype, dev):
        """Persistent packed-weight buffer (re-used every step, so the batched pack's job
        table stays valid); zero-filled once, so the padding a padded pack skips stays zero."""
        t = self._bufs.get(name)
        if t is None or t.numel() != n or t.dtype != dtype or t.device != dev:
            t = self._bufs[name] = torch.zeros(n, device=dev, dtype=dtype)
        return t

    def pack(self):
        """Weights in kernel layouts (bf16 / fp32 pointwise [co][ci], depthwise taps [9][C],
        conv2 [co][tap][ci]), all repacked by one batched launch when a parameter changed."""
        key = self._version_key()
        if key == self._pack_key:
            return self._packed
        dt, pk, jobs = self.dtype, {}, []
        m = self.model
        dev = m.conv1.weight.device

        def add(name, w, n_dtype, d0, d1, d2, perm, rows=None, pitch=None):
            """pack w permuted; rows x pitch: padded [rows][pitch] destination (2-D packs)"""
            n = rows * pitch if rows else d0 * d1 * d2
            out = self._buf(name, n, n_dtype, dev)
            jobs.append((w.detach(), out, d0, d1, d2, perm, pitch))
            pk[name] = out

        for u in self._all_units():
            c = u.sep.conv1.in_channels
            add(u.name + ".dw", u.sep.conv1.weight, torch.float32, c, 9, 1, (1, 0, 2), 9, pc(c))
            pw = u.sep.pointwise
            co, ci = pw.out_channels, pw.in_channels
            add(u.name + ".pw", pw.weight, dt, co, ci, 1, (0, 1, 2), pc(co), pc(ci))
        for b in self.blocks:
            if b.skip is not None:
                co, ci = b.skip.out_channels, b.skip.in_channels
                add(b.name + ".skip", b.skip.weight, dt, co, ci, 1, (0, 1, 2), pc(co), pc(ci))
        add("conv2", m.conv2.weight, dt, 64, 32, 9, (0, 2, 1))   # [co][tap][ci]
        self._pack_fwd.run(jobs)
        self._packed, self._pack_key = pk, key
        self._packed_bwd_key = None
        return pk

    def pack_bwd(self):
        """Transposed weights for the input-gradient GEMMs (one batched launch)."""
        if self._packed_bwd_key == self._pack_key and self._pack_key is not None:
            return self._packed
        pk, dt, m = self._packed, self.dtype, self.model
        dev = m.conv1.weight.device
        jobs = []

        def add(name, w, d0, d1, d2, perm, rows=None, pitch=None):
            n = rows * pitch if rows else d0 * d1 * d2
            out = self._buf(name, n, dt, dev)
            jobs.append((w.detach(), out, d0, d1, d2, perm, pitch))
            pk[name] = out

        for u in self._all_units():
            pw = u.sep.pointwise
            co, ci = pw.out_channels, pw.in_channels
            add(u.name + ".pwT", pw.weight, co, ci, 1, (1, 0, 2), pc(ci), pc(co))
        for b in self.blocks:
            if b.skip is not None:
                co, ci = b.skip.out_channels, b.skip.in_channels
                add(b.name + ".skipT", b.skip.weight, co, ci, 1, (1, 0, 2), pc(ci), pc(co))
        add("conv2T", m.conv2.weight, 64, 32, 9, (1, 2, 0))   # [ci][tap][co]
        self._pack_bwd.run(jobs)
        self._packed_bwd_key = self._pack_key
        return pk

    def _all_units(self):
        for b in self.blocks:
            yield from b.units
        yield from self.exit_units

    # ------------------------------------------------------------ helpers
    def _empty(self, n, dtype=None):
        return torch.empty(n, device=self.device, dtype=dtype or self.dtype)

    def _bn_stats(self, part, R, C, count, bnmod, train):
        """BN statistics of a C-channel tensor (partials and Stats at its channel pitch)"""
        CP = pc(C)
        s = Stats(CP, self.device)
        ref = _bn_ref(bnmod)
        self.model._xcp_wait_buffers()   # a buffer broadcast still in flight (xcp.ddp.broadcast_buffers)
        if train:
            if ref["momentum"] is None:
                ref["momentum"] = 1.0 / float(bnmod.num_batches_tracked.item() + 1)
            ops.finalize_stats(part, R, C, count, ref, True, s, CP)
        else:
            ops.eval_stats(C, ref, s, self.device, CP)
        return s

    def _pw(self, A, Wp, M, cout, cin, train, bnmod, lda=None, gather=(0, 0, 0, 0, 0, 1, 0)):
        """pointwise conv at the channel pitches (padded output channels come out zero)"""
        cop, cip = pc(cout), pc(cin)
        Y = self._empty(M * cop)
        if train:
            R = ops.nt_stat_rows(M)
            part = self._empty(R * 2 * cop, torch.float32)
            ops.gemm_nt(A, Wp, Y, M, cop, cip, lda=lda, stats=part, gather=gather, tile=NT_TILE)
            st = self._bn_stats(part, R, cout, M, bnmod, True)
        else:
            ops.gemm_nt(A, Wp, Y, M, cop, cip, lda=lda, gather=gather, tile=NT_TILE)
            st = self._bn_stats(None, 0, cout, M, bnmod, False)
        return Y, st

    # ------------------------------------------------------------ forward
    def forward(self, x, train):
        """x: [N,3,H,W] fp32 (NCHW, as XceptionLSTMV.extract_features feeds it).
        Returns (features [N,2048] fp32, saved-state dict for backward)."""
        ops.check_gpu(x)
        with ops.device_guard(x):
            return self._forward(x, train)

    def _forward(self, x, train):
        self.device = x.device
        x = x.contiguous().float()
        N, C0, IH, IW = x.shape
        if C0 != 3:
            raise ValueError("Xception expects 3 input channels")
        pk = self.pack()
        m = self.model
        S = {"N": N, "IH": IH, "IW": IW, "x": x, "train": train}
        # ---- stem (Xception.py:168-174)
        OH1, OW1 = (IH - 3) // 2 + 1, (IW - 3) // 2 + 1
        rows1 = N * OH1 * OW1
        c1 = self._empty(rows1 * 32)
        if train and CONV1_STATS_FUSED and ops.conv1_wgrad_fused(self.dtype, IH, IW):
            part, R = ops.conv1_fwd_stats(x, m.conv1.weight.detach(), c1, N, IH, IW)
            s1 = self._bn_stats(part, R, 32, rows1, m.bn1, True)
        elif train:
            ops.conv1_fwd(x, m.conv1.weight.detach(), c1, N, IH, IW)
            part, R = ops.row_stats(c1, rows1, 32)
            s1 = self._bn_stats(part, R, 32, rows1, m.bn1, True)
        else:
            ops.conv1_fwd(x, m.conv1.weight.detach(), c1, N, IH, IW)
            s1 = self._bn_stats(None, 0, 32, rows1, m.bn1, False)
        OH2, OW2 = OH1 - 2, OW1 - 2
        rows2 = N * OH2 * OW2
        R2 = ops.conv3x3_parts(0, N, OH1, OW1) if self.dtype == torch.bfloat16 else 0
        # conv2 and its weight gradient apply BN1 + ReLU to conv1's output as they stage it: a1 =
        # relu(bn1(c1)) is never written (CONV2_ACT_ON_LOAD)
        act_on_load = CONV2_ACT_ON_LOAD and R2 > 0 and (not train or ops.conv3x3_wgrad_parts(N, OH1, OW1) > 0)
        if act_on_load:
            a1 = None
        else:
            a1 = self._empty(rows1 * 32)
            ops.bn_act(c1, a1, s1.scale, s1.shift, True, rows1, 32)
        if R2 > 0:   # direct MFMA conv (conv3.hip)
            c2 = self._empty(rows2 * 64)
            part = self._empty(R2 * 2 * 64, torch.float32) if train else None
            if act_on_load:
                ops.conv3x3(0, c1, pk["conv2"], c2, part, N, OH1, OW1, in_scale=s1.scale, in_shift=s1.shift)
            else:
                ops.conv3x3(0, a1, pk["conv2"], c2, part, N, OH1, OW1)
            s2 = self._bn_stats(part, R2, 64, rows2, m.bn2, train)
        else:        # implicit GEMM (im2col gather)
            c2, s2 = self._pw(a1, pk["conv2"], rows2, 64, 288, train, m.bn2, lda=32,
                              gather=(2, OH1, OW1, OH2, OW2, 1, 32))
        S.update(c1=c1, s1=s1, a1=a1, c2=c2, s2=s2, OH1=OH1, OW1=OW1, OH2=OH2, OW2=OW2)
        # ---- blocks (Xception.py:176-187)
        S["blocks"] = []
        b0 = self.blocks[0]
        if STEM_FUSED and not b0.units[0].relu and b0.skip is not None and b0.stride != 1:
            # block1 (start_with_relu=False, stride-2 skip conv): x = relu(bn2(conv2)) is never
            # materialised at 147^2 -- the first depthwise conv applies BN2 + ReLU on load and the
            # skip conv reads only the stride-2 pixels, activated by one small pass
            OHs, OWs = (OH2 - 1) // b0.stride + 1, (OW2 - 1) // b0.stride + 1
            skip_x = self._empty(N * OHs * OWs * 64)
            ops.bn_act_strided(c2, skip_x, s2.scale, s2.shift, True, N, OH2, OW2, OHs, OWs, b0.stride, 64)
            xc, H, W, bs = self._block_fwd(b0, c2, N, OH2, OW2, pk, train, pre_bn=s2, skip_x=skip_x)
            S["blocks"].append(bs)
            rest = self.blocks[1:]
        else:
            xc = self._empty(rows2 * 64)
            ops.bn_act(c2, xc, s2.scale, s2.shift, True, rows2, 64)
            H, W, rest = OH2, OW2, self.blocks
        for b in rest:
            xc, H, W, bs = self._block_fwd(b, xc, N, H, W, pk, train)
            S["blocks"].append(bs)
        # ---- exit flow (Xception.py:189-198)
        M = N * H * W
        ex = []
        src, act, sc, sh = xc, ACT_NONE, None, None
        for u in self.exit_units:
            d = self._empty(M * pc(u.cin))
            ops.dw_fwd(act, src, d, pk[u.name + ".dw"], sc, sh, N, H, W, pc(u.cin))
            y, st = self._pw(d, pk[u.name + ".pw"], M, u.cout, u.cin, train, u.bn)
            ex.append({"src": src, "act": act, "sc": sc, "sh": sh, "d": d, "y": y, "st": st})
            src, act, sc, sh = y, ACT_BNRELU, st.scale, st.shift
        feats = torch.empty(N, 2048, device=self.device, dtype=torch.float32)
        last = ex[-1]
        ops.avgpool_fwd(last["y"], last["st"].scale, last["st"].shift, feats, N, H * W, 2048)
        S.update(exit=ex, xH=H, xW=W, x12=xc)
        if train:
            nbt = [b.num_batches_tracked for b in self.bn_modules if b.num_batches_tracked is not None]
            if nbt:
                torch._foreach_add_(nbt, 1)
        return feats, S

    def _block_fwd(self, b, x_in, N, H, W, pk, train, pre_bn=None, skip_x=None):
        """pre_bn: Stats of a BN + ReLU the block's input still needs (applied on load by the first
        depthwise conv); skip_x: the skip conv's input, already strided and activated"""
        if pre_bn is not None and (b.skip is None or b.stride == 1 or b.units[0].relu):
            raise ValueError("pre_bn: only a block without a leading ReLU and with a strided skip conv")
        M = N * H * W
        units = []
        src, act, sc, sh = x_in, (ACT_RELU if b.units[0].relu else ACT_NONE), None, None
        if pre_bn is not None:
            act, sc, sh = ACT_BNRELU, pre_bn.scale, pre_bn.shift
        for u in b.units:
            d = self._empty(M * pc(u.cin))
            R = (ops.sep_fwd_parts(self.dtype, N, H, W, u.cin, u.cout)
                 if SEP_FUSED and train and pc(u.cin) == u.cin and pc(u.cout) == u.cout
                 and W >= SEP_MIN_W.get(u.cout, 1 << 30) else 0)
            if R > 0:
                y = self._empty(M * u.cout)
                part = self._empty(R * 2 * u.cout, torch.float32)
                ops.sep_fwd(act, src, sc, sh, pk[u.name + ".dw"], pk[u.name + ".pw"], d, y, part, N, H, W, u.cin, u.cout)
                st = self._bn_stats(part, R, u.cout, M, u.bn, True)
            else:
                ops.dw_fwd(act, src, d, pk[u.name + ".dw"], sc, sh, N, H, W, pc(u.cin))
                y, st = self._pw(d, pk[u.name + ".pw"], M, u.cout, u.cin, train, u.bn)
            units.append({"src": src, "act": act, "sc": sc, "sh": sh, "d": d, "y": y, "st": st})
            src, act, sc, sh = y, ACT_BNRELU, st.scale, st.shift
        if b.pool or b.stride != 1:
            OH, OW = (H - 1) // b.stride + 1, (W - 1) // b.stride + 1
        else:
            OH, OW = H, W
        Ms = N * OH * OW
        ys = sks = None
        if b.skip is not None and skip_x is not None:
            ys, sks = self._pw(skip_x, pk[b.name + ".skip"], Ms, b.cout, b.cin, train, b.skipbn, lda=pc(b.cin))
        elif b.skip is not None:
            ys, sks = self._pw(x_in, pk[b.name + ".skip"], Ms, b.cout, b.cin, train, b.skipbn, lda=pc(b.cin),
                               gather=(1, H, W, OH, OW, b.stride, 0) if b.stride != 1 else (0, 0, 0, 0, 0, 1, 0))
        out = self._empty(Ms * pc(b.cout))
        amax = torch.empty(Ms * pc(b.cout), device=self.device, dtype=torch.uint8) if b.pool else None
        st = units[-1]["st"]
        ops.tail_fwd(units[-1]["y"], st.scale, st.shift, b.pool, ys if ys is not None else x_in,
                     sks.scale if sks is not None else None, sks.shift if sks is not None else None, out, amax, N, H, W,
                     pc(b.cout))
        bs = {"x_in": x_in, "units": units, "ys": ys, "sks": sks, "amax": amax, "H": H, "W": W, "OH": OH, "OW": OW,
              "pre_bn": pre_bn, "skip_x": skip_x}
        return out, OH, OW, bs

    # ------------------------------------------------------------ backward
    def backward(self, S, dfeat, out=None, notify=None):
        """dfeat [N,2048] fp32 -> backbone parameter gradients.

        out None: returns {param name: fresh fp32 gradient}.  out {name: tensor}: the
        gradients of those parameters are ADDED to the given tensors (param.grad views);
        others are returned fresh.  notify(names, side_stream): called after the kernels
        that produce the gradients of ``names`` are enqueued (side_stream: the stream the
        weight gradients run on, or None)."""
        if not S["train"]:
            raise RuntimeError("xcp engine backward needs a train-mode forward (batch-stat BatchNorm)")
        with ops.device_guard(dfeat):
            return self._backward(S, dfeat, out, notify)

    def _backward(self, S, dfeat, out, notify):
        pk = self.pack_bwd()
        m = self.model
        N = S["N"]
        dev = self.device
        grads = {}
        dfeat = dfeat.contiguous().float()
        out = out or {}
        pending = []

        def g(name, shape):
            """(gradient tensor of parameter ``name``, accumulate into it?)"""
            pending.append(name)
            t = out.get(name)
            if t is not None:
                return t, True
            t = torch.empty(shape, device=dev, dtype=torch.float32)
            grads[name] = t
            return t, False

        # Pointwise weight gradients run on a side stream: they depend only on dY (and a saved
        # activation), nothing downstream waits for them until the backward returns, so they
        # overlap the dgrad GEMMs and depthwise backward kernels of the main stream.
        main = torch.cuda.current_stream(dev)
        side = self._side_stream(dev) if WGRAD_SIDE_STREAM else None
        # Main-stream tensors the side stream reads are kept referenced here until the main
        # stream has waited for the side stream (end of this backward); freeing them after that
        # point is stream-ordered, so the caching allocator may hand them out again at once.
        # (record_stream instead defers their reuse until the side stream's work has actually
        # run on the GPU; with the host a step or more ahead of the GPU that kept every step's
        # backward temporaries unusable and the allocator mapped fresh device memory every step:
        # 140-170 hipMallocs in 20 timed steps and 149 GB reserved for 25.6 GB in use.)
        keep = []
        # the weight-gradient slab reductions of one block (pointwise split-K slabs, depthwise
        # partials) go out together in one or two launches when the block is done (REDUCE_BATCH)
        rbatch = ops.ReduceBatch() if REDUCE_BATCH else None

        deferred = []   # (WGRAD_DEFER) the last unit's weight gradient, launched after the next input gradient

        def wgrad(G, X, M, Nn, K, name, shape, defer=False, **kw):
            """dW[Nn][K] = G^T X (logical channels; G / X at their channel pitches)"""
            kw.setdefault("ldg", pc(Nn))
            kw.setdefault("ldx", pc(K))
            dst, acc = g(name, shape)
            if side is None:
                ops.weight_grad(G, X, M, Nn, K, dst, accumulate=acc, batch=rbatch, **kw)
                return
            if defer:
                flush_deferred()
                deferred.append((G, X, M, Nn, K, dst, acc, kw))
                keep.extend((G, X))
                return
            side.wait_stream(main)
            with torch.cuda.stream(side):
                ops.weight_grad(G, X, M, Nn, K, dst, accumulate=acc, batch=rbatch, **kw)
            keep.extend((G, X))   # dst: a gradient, referenced by the caller until the end

        def flush_deferred():
            if deferred:
                side.wait_stream(main)
                with torch.cuda.stream(side):
                    for G, X, M, Nn, K, dst, acc, kw in deferred:
                        ops.weight_grad(G, X, M, Nn, K, dst, accumulate=acc, batch=rbatch, **kw)
                deferred.clear()

        def done():
            """every gradient requested since the last call is enqueued: reduce the block's slabs,
            tell the sink"""
            flush_deferred()
            if rbatch is not None and rbatch.jobs:
                if side is not None:
                    side.wait_stream(main)   # the depthwise partials come from the main stream
                    with torch.cuda.stream(side):
                        rbatch.flush()
                else:
                    rbatch.flush()
            if notify is not None and pending:
                notify(list(pending), side)
            pending.clear()

        def bn_coef(bnmod, name, dZ, Y, rows, C, st, part=None, relu=False, narrow=False):
            """BN backward up to its coefficients (alpha, bcoef, delta; at the channel pitch);
            writes the affine grads"""
            P = part[1] if part is not None else 0
            (gw, acc), (gb, acc_b) = g(name + ".weight", (C,)), g(name + ".bias", (C,))
            if acc != acc_b:
                raise NotImplementedError(f"xcp engine: {name}.weight and .bias must both (or neither) require grad")
            return ops.bn_backward_coef(dZ, Y, rows, C, _bn_ref(bnmod), st, gw, gb,
                                        part=part[0] if part is not None else None, R=P, relu=relu, accumulate=acc,
                                        CP=pc(C), narrow=narrow)

        def bn_bwd(bnmod, name, dZ, Y, rows, C, st, part=None, relu=False):
            coef = bn_coef(bnmod, name, dZ, Y, rows, C, st, part, relu)
            dY = self._empty(rows * pc(C))
            ops.bn_apply_coef(dZ, Y, dY, coef, st, rows, pc(C), relu)
            return dY

        def unit_bwd(u, rec, dZ, H, W, dRes=None, dSkip=None, skip_geom=(0, 0, 1), part=None, prev_st=None,
                     skip_pre=False, res_bn=None):
            """dZ: gradient w.r.t. this unit's BN output (``part``: its fused BN-backward
            partial sums, if the producer emitted them).  Returns (gradient w.r.t. the
            depthwise input after the activation mask (+ residual / skip terms), and -- when
            ``prev_st`` is the Stats of the BN feeding this unit -- that BN's backward partial
            sums)."""
            M = N * H * W
            dD = self._empty(M * pc(u.cin))
            if FUSED_UNIT_BWD and ops.unit_bwd_rows_per_split(dZ.dtype, M, u.cout, u.cin) > 0:
                # narrow units: BN apply + pointwise dgrad + wgrad in one pass (dY stays on chip)
                coef = bn_coef(u.bn, u.bn_name, dZ, rec["y"], M, u.cout, rec["st"], part)
                dst, acc = g(u.name + ".pointwise.weight", (u.cout, u.cin, 1, 1))
                ops.unit_bwd(dZ, rec["y"], coef, pk[u.name + ".pwT"], rec["d"], dD, M, u.cout, u.cin, dst, acc)
            else:
                dY = bn_bwd(u.bn, u.bn_name, dZ, rec["y"], M, u.cout, rec["st"], part)
                if WGRAD_FIRST:   # the side stream starts on dY before this unit's input gradient (A/B)
                    wgrad(dY, rec["d"], M, u.cout, u.cin, u.name + ".pointwise.weight", (u.cout, u.cin, 1, 1))
                ops.gemm_nt(dY, pk[u.name + ".pwT"], dD, M, pc(u.cin), pc(u.cout), tile=NT_TILE)
                if not WGRAD_FIRST:
                    wgrad(dY, rec["d"], M, u.cout, u.cin, u.name + ".pointwise.weight", (u.cout, u.cin, 1, 1),
                          defer=WGRAD_DEFER)
            dX = self._empty(M * pc(u.cin))
            dwg, acc = g(u.name + ".conv1.weight", (u.cin, 1, 3, 3))
            bnp = ops.dw_bwd(rec["act"], dD, rec["src"], pk[u.name + ".dw"], rec["sc"], rec["sh"], dX, dwg, N, H, W,
                             pc(u.cin), dRes=dRes, dSkip=dSkip, skip_geom=skip_geom,
                             bn_stats=res_bn[1] if res_bn is not None else prev_st, accumulate=acc,
                             Cw=u.cin, skip_pre=skip_pre, reduce_stream=side if DW_REDUCE_SIDE else None,
                             keep=keep, batch=rbatch, res_bn_input=res_bn[0] if res_bn is not None else None)
            return dX, (bnp if prev_st is not None or res_bn is not None else None)

        # ---- exit flow
        H, W = S["xH"], S["xW"]
        M = N * H * W
        e3, e4 = S["exit"]
        u3, u4 = self.exit_units
        dZ4 = self._empty(M * 2048)
        ops.avgpool_bwd(dfeat, e4["y"], e4["st"].scale, e4["st"].shift, dZ4, N, H * W, 2048)
        dZ3, p3 = unit_bwd(u4, e4, dZ4, H, W, prev_st=e3["st"])
        dX, _ = unit_bwd(u3, e3, dZ3, H, W, part=p3)
        done()
        # ---- blocks, last to first
        pre_part = part_in = None
        for k in range(len(self.blocks) - 1, -1, -1):
            prev = (self.blocks[k - 1], S["blocks"][k - 1]) if k > 0 else None
            dX, pre_part, part_in = self._block_bwd(self.blocks[k], S["blocks"][k], dX, N, pk, bn_bwd, unit_bwd,
                                                    wgrad, part_in, prev)
            done()
        # ---- stem
        OH1, OW1, OH2, OW2 = S["OH1"], S["OW1"], S["OH2"], S["OW2"]
        rows1, rows2 = N * OH1 * OW1, N * OH2 * OW2
        if pre_part is not None:   # block1 applied BN2 + ReLU on load: dX is masked, its BN2 sums came along
            dC2 = bn_bwd(m.bn2, "bn2", dX, S["c2"], rows2, 64, S["s2"], part=pre_part)
        else:
            dC2 = bn_bwd(m.bn2, "bn2", dX, S["c2"], rows2, 64, S["s2"], relu=True)   # relu (Xception.py:174) fused
        def conv2_wgrad(st2):
            """conv2's weight gradient (from dC2 and a1) on stream st2 (None: the current one)"""
            if st2 is not None:
                st2.wait_stream(main)
            c2g, acc = g("conv2.weight", (64, 32, 3, 3))   # (allocated on the main stream)
            with torch.cuda.stream(st2) if st2 is not None else contextlib.nullcontext():
                w2g = torch.empty(64 * 288, device=dev, dtype=torch.float32)
                if S["a1"] is None:   # (conv2 read conv1's output with BN1 + ReLU on load)
                    ops.conv3x3_wgrad(dC2, S["c1"], w2g, N, OH1, OW1, in_scale=S["s1"].scale, in_shift=S["s1"].shift)
                elif self.dtype == torch.bfloat16 and ops.conv3x3_wgrad_parts(N, OH1, OW1) > 0:
                    ops.conv3x3_wgrad(dC2, S["a1"], w2g, N, OH1, OW1)
                else:
                    ops.weight_grad(dC2, S["a1"], rows2, 64, 288, w2g, gather=(2, OH1, OW1, OH2, OW2, 1, 32), ldx=32)
                if acc:
                    tmp = torch.empty_like(c2g)
                    ops.permute3(w2g, tmp, 64, 9, 32, (0, 2, 1))
                    c2g.add_(tmp)
                else:
                    ops.permute3(w2g, c2g, 64, 9, 32, (0, 2, 1))
            if st2 is not None:
                keep.append(dC2)

        st2 = side if STEM_WGRAD_SIDE else None
        if STEM_WGRAD_EARLY and st2 is not None:   # beside conv2's input gradient (A/B)
            conv2_wgrad(st2)
        dA1 = self._empty(rows1 * 32)
        if self.dtype == torch.bfloat16 and ops.conv3x3_parts(1, N, OH2, OW2) > 0:
            ops.conv3x3(1, dC2, pk["conv2T"], dA1, None, N, OH2, OW2)
        else:
            ops.gemm_nt(dC2, pk["conv2T"], dA1, rows1, 32, 576, lda=64, gather=(3, OH1, OW1, OH2, OW2, 1, 64))
        # BN1's backward coefficients first (per-channel reduce + finalize on the main stream), then
        # conv2's weight gradient on the weight-gradient stream beside the rest of the chain (BN1
        # apply, conv1's weight gradient).  Launched the other way round, the finalize's one
        # 1024-thread workgroup waited for the side stream's conv2 weight gradient to leave the CUs:
        # 356 us per step on the main stream (profiles/r03_v3_kernels.txt)
        # (narrow finalize: conv2's weight gradient holds every CU beside it when launched early)
        if STEM_BN1_FIRST:
            coef1 = bn_coef(m.bn1, "bn1", dA1, S["c1"], rows1, 32, S["s1"], None, True,   # relu (Xception.py:170)
                            narrow=STEM_FIN_NARROW and STEM_WGRAD_EARLY and st2 is not None)
        if not (STEM_WGRAD_EARLY and st2 is not None):
            conv2_wgrad(st2)
        if not STEM_BN1_FIRST:
            coef1 = bn_coef(m.bn1, "bn1", dA1, S["c1"], rows1, 32, S["s1"], None, True)
        c1g, acc = g("conv1.weight", (32, 3, 3, 3))
        if CONV1_BN_FUSED and pc(32) == 32 and ops.conv1_wgrad_fused(self.dtype, S["IH"], S["IW"]):
            ops.conv1_wgrad_bn(S["x"], dA1, S["c1"], coef1, S["s1"], c1g, N, S["IH"], S["IW"], 32, relu=True,
                               accumulate=acc)
        else:
            dC1 = self._empty(rows1 * pc(32))
            ops.bn_apply_coef(dA1, S["c1"], dC1, coef1, S["s1"], rows1, pc(32), relu=True)
            ops.conv1_wgrad(S["x"], dC1, c1g, N, S["IH"], S["IW"], accumulate=acc)
        if side is not None:
            main.wait_stream(side)
        keep.clear()   # after the wait: reuse of these blocks is ordered behind the side stream
        done()
        return grads

    def _block_bwd(self, b, bs, dOut, N, pk, bn_bwd, unit_bwd, wgrad, part_in=None, prev=None):
        """part_in: partial sums of this block's last BN (whose output gradient is dOut), produced by
        the next block's first depthwise backward; prev: (block, forward state) of the block before.
        Returns (gradient w.r.t. the block input, the stem BN2 partials (block1 only), the partial sums
        of prev's last BN when this block's first depthwise backward produced them)."""
        H, W, OH, OW = bs["H"], bs["W"], bs["OH"], bs["OW"]
        Ms = N * OH * OW
        units = bs["units"]
        # pooled block: one pass materialises the max-pool gradient (per-quad gather) and
        # reduces it for the last unit's BN backward (1.50 vs 1.58 ms with a separate reduce
        # at 147^2 x 128; gathering it inside the BN-backward kernels measured 1.83 / 1.88 ms)
        part = None if b.pool else part_in   # (a pooled tail's backward reduces its last BN itself)
        if b.pool:
            dZ = self._empty(N * H * W * pc(b.cout))
            part = ops.maxpool_bwd_bnred(dOut, bs["amax"], dZ, units[-1]["y"], units[-1]["st"], N, H, W, pc(b.cout))
        else:
            dZ = dOut
        dRes = dSkip = None
        skip_geom = (0, 0, 1)
        if b.skip is not None:
            dYs = bn_bwd(b.skipbn, b.name + ".skipbn", dOut, bs["ys"], Ms, b.cout, bs["sks"])

            def skip_wgrad():
                if bs["skip_x"] is not None:
                    wgrad(dYs, bs["skip_x"], Ms, b.cout, b.cin, b.name + ".skip.weight", (b.cout, b.cin, 1, 1))
                else:
                    wgrad(dYs, bs["x_in"], Ms, b.cout, b.cin, b.name + ".skip.weight", (b.cout, b.cin, 1, 1),
                          gather=(1, H, W, OH, OW, b.stride, 0) if b.stride != 1 else (0, 0, 0, 0, 0, 1, 0))
            if not SKIP_WGRAD_LATE:
                skip_wgrad()
            dXs = self._empty(Ms * pc(b.cin))
            ops.gemm_nt(dYs, pk[b.name + ".skipT"], dXs, Ms, pc(b.cin), pc(b.cout), tile=NT_TILE)
            if b.stride != 1:
                dSkip, skip_geom = dXs, (OH, OW, b.stride)
            else:
                dRes = dXs
        else:
            dRes = dOut
        for i in range(len(b.units) - 1, -1, -1):
            u, rec = b.units[i], units[i]
            if i > 0:
                dZ, part = unit_bwd(u, rec, dZ, H, W, part=part, prev_st=units[i - 1]["st"])
            else:
                pre = bs["pre_bn"]
                # identity-skip boundary: prev's output is BN(y) + its input (no pool after the BN), so
                # this unit's final dX is the gradient w.r.t. that BN's output
                res_bn = None
                if (RESBN and pre is None and dRes is not None and dSkip is None and prev is not None
                        and not prev[0].pool):
                    last = prev[1]["units"][-1]
                    res_bn = (last["y"], last["st"])
                dZ, out_part = unit_bwd(u, rec, dZ, H, W, dRes=dRes, dSkip=dSkip, skip_geom=skip_geom, part=part,
                                        prev_st=pre, skip_pre=pre is not None, res_bn=res_bn)
                pre_part = out_part if pre is not None else None
                prev_part = out_part if res_bn is not None else None
        if b.skip is not None and SKIP_WGRAD_LATE:
            skip_wgrad()
        return dZ, pre_part, prev_part


class XceptionFunction(torch.autograd.Function):
    """Autograd node for the whole backbone: inputs (frames, *backbone params),
    output features [N,2048].  Gradients w.r.t. the frames are not produced (the
    reference never differentiates w.r.t. its input clips)."""

    @staticmethod
    def forward(ctx, engine, train, x, *params):
        feats, S = engine.forward(x, train)
        ctx.engine, ctx.S = engine, S
        ctx.names = [n for n, _ in engine.named_params()]
        ctx.needs = [p.requires_grad for p in params]
        ctx.params = params
        return feats

    @staticmethod
    def backward(ctx, dfeat):
        eng = ctx.engine
        sink = eng.grad_sink
        need = {n for n, nd in zip(ctx.names, ctx.needs) if nd}
        if sink is None:
            # default: hand the gradients to autograd (hooks and autograd.grad behave as usual)
            grads = eng.backward(ctx.S, dfeat)
            ctx.S = ctx.params = None
            return (None, None, None, *[grads.get(n) if n in need else None for n in ctx.names])
        # gradient sink: accumulate straight into the sink's param.grad views, block by block
        out = {}
        for n, p in zip(ctx.names, ctx.params):
            if n in need:
                # the sink's flat view (re-attached, zeroed, after optimizer.zero_grad() set it to
                # None), so what the kernels add is what the bucket all-reduce sees
                out[n] = sink.grad_view(p)
        by_name = dict(zip(ctx.names, ctx.params))
        eng.backward(ctx.S, dfeat, out=out,
                     notify=lambda names, side: sink.ready([by_name[n] for n in names if n in need], side))
        ctx.S = ctx.params = None
        return (None, None, None, *([None] * len(ctx.names)))
