"""One-process-per-GPU data parallelism for the clip models (RCCL over xGMI).

Replaces the reference's single-process ``nn.DataParallel`` (train_audio.py:16-18,
which also bypasses DP for the backbone, :37).  Every rank owns a full replica
and a shard of the clip minibatch; the only exchange per step is the gradient
mean, done here as bucketed ``all_reduce`` calls (``"nccl"`` = RCCL on ROCm) on
one flat fp32 gradient buffer that the parameters' ``.grad`` tensors are views
of.  BatchNorm statistics stay per rank (the reference has no SyncBN); running
buffers are broadcast from rank 0 before each forward (DDP ``broadcast_buffers``
semantics).

Overlap with backward.  Parameters sit in the flat buffer in reverse registration
order, which is the order backward produces their gradients (head first, then the
backbone from the exit flow down to the stem), and buckets are contiguous ranges of
it.  A bucket's all-reduce is launched the moment its last gradient is final:

* head parameters (LSTM / FC) report through post-accumulate-grad hooks;
* backbone parameters report through the xcp engine's gradient sink
  (``module=`` registers this object with every Xception engine inside the model):
  the engine accumulates straight into the ``.grad`` views and calls ``ready`` after
  each block, so the buckets of blocks 12 ... k are reduced while blocks k-1 ... 1
  are still in backward.

Streams.  A bucket's gradients are written by the main (backward) stream and, for the
pointwise weight gradients, by the engine's weight-gradient side stream.  A completed bucket's
all-reduce is launched from the side stream after it waits on the main stream (which it is
normally behind already): the collective then follows every gradient of the bucket, and the main
stream never waits on the side stream or on a collective before the backward has been enqueued
(``allreduce()`` makes it wait for the collectives, the engine for its side stream at the end of
its backward).  Making the main stream wait on the side stream at every completed bucket instead
(round 3) would drain the side stream's queued weight-gradient GEMMs mid-backward, about once per
25 MB bucket, and give back the overlap the side stream exists for.  A third, dedicated
communication stream waiting on both was measured and dropped (XCP_DDP_LAUNCH above).

The mean is formed inside the collective: ``ReduceOp.AVG`` on RCCL (``"nccl"``), so no extra pass
over the 100.8 MB buffer follows the reduction; gloo (the CPU tests) has no AVG and keeps SUM plus
one scaling pass per bucket.

Buffers.  ``broadcast_buffers`` launches rank 0's BatchNorm running statistics from a stream of its
own (one persistent flat buffer: gather, broadcast, scatter back) and hands the completion event to
every xcp Xception backbone in the module; the main stream waits on it only where the forward first
reads or writes a running statistic (the stem's BN1 statistics, after conv1 has been enqueued -- on
the fused engine and on the module path alike), not before the step starts.  ``state_dict()``,
pickling and DataParallel replication wait too; other readers call ``wait_buffers(module)``.  That is the RCCL form; under gloo (whose wait() blocks the host until the
side stream has drained) the broadcast completes on the current stream.

Which parameters take part is re-read at every ``zero()``: the reference trains with
the backbone frozen for three epochs and then unfreezes it (train_visual.py:547-556);
frozen parameters keep ``grad = None`` (so an optimiser skips them, as in the reference)
and buckets only span parameters that require grad.
"""
import os
import weakref

import torch
import torch.distributed as dist

# Where a bucket's all-reduce is launched from (XCP_DDP_LAUNCH):
#   side (default): the engine's weight-gradient stream, after it waits on the current stream;
#   comm: a communication stream of its own that waits on both (measured: the 2-rank gloo path ran
#         13-17x slower per step this way, 944 vs 74 ms at 4 clips per rank, profiles/r04_ddp_ab.txt);
#   main: the current stream after it waits on the weight-gradient stream (the round-3 order).
DDP_LAUNCH = os.environ.get("XCP_DDP_LAUNCH", "side")
if DDP_LAUNCH not in ("side", "comm", "main"):
    raise ValueError("XCP_DDP_LAUNCH must be side, comm or main")


class GradBuckets:
    def __init__(self, params, bucket_bytes=25 << 20, world=None, module=None, proxy=None):
        """proxy (one GPU, world size 1 only): {"world": G, "busbw": GB/s, "blocks": n} launches, at each
        bucket-ready point and from the same stream a real all-reduce would start on, a stand-in of
        RCCL's footprint (xcp_comm_proxy: n workgroups stream the bucket once and hold their CUs for
        2 (G - 1) / G x bytes / busbw) and stamps the ready point, each stand-in's first / last
        workgroup start and end and the backward's end on one clock (proxy_report()).  It measures
        whether the collectives would start while the weight-gradient stream holds the CUs and how
        much of them would be left after the backward (profiles/r06_ddp_proxy.txt)."""
        self.params = list(params)
        if not self.params:
            raise ValueError("GradBuckets: no parameters")
        self.world = world if world is not None else (dist.get_world_size() if dist.is_initialized() else 1)
        self.bucket_elems = max(1, bucket_bytes // 4)
        dev = self.params[0].device
        # every view starts on a 16-B boundary (slots padded to 4 floats, the padding stays zero):
        # the batched slab reductions write float4 lanes straight into the .grad views
        slot = lambda n: (n + 3) // 4 * 4   # noqa: E731
        self.flat = torch.zeros(sum(slot(p.numel()) for p in self.params), device=dev, dtype=torch.float32)
        self.views = {}
        self._slot = {}
        off = 0
        for p in reversed(self.params):   # backward order
            self.views[p] = (off, p.numel())
            self._slot[p] = slot(p.numel())
            off += self._slot[p]
        self.proxy = dict(proxy) if proxy and self.world == 1 and dev.type == "cuda" else None
        self.overlap = self.world > 1 or self.proxy is not None
        self.sync = True   # False: gradient accumulation micro-batch, no all-reduce launched
        self._active_key = None
        self._pending = []
        self._hooked = set()
        self._comm = None
        self.use_streams = dev.type == "cuda"
        # average inside the collective where the backend has it (RCCL); gloo: SUM, then scale
        self.avg = dist.is_initialized() and dist.get_backend() == "nccl"
        if module is not None:
            self.attach(module)
        if self.proxy is not None:
            self._prx_step = -1
            self._prx_scratch = torch.empty_like(self.flat)
        self.zero()

    # ------------------------------------------------------------ layout
    def attach(self, module):
        """Register as the gradient sink of every xcp Xception backbone inside ``module``."""
        for m in module.modules():
            if hasattr(m, "_xcp_grad_sink"):
                m._xcp_grad_sink = self

    def _layout(self):
        """Buckets over the parameters that currently require grad: contiguous runs of the flat
        buffer, split at bucket_elems."""
        active = [p for p in reversed(self.params) if p.requires_grad]
        self.active = active
        self.buckets, self._bucket_of = [], {}
        cur, start, end = [], None, None
        for p in active:
            o, _ = self.views[p]
            n = self._slot[p]
            if cur and (o != end or end - start + n > self.bucket_elems):
                self.buckets.append((start, end, cur))
                cur = []
            if not cur:
                start = o
            cur.append(p)
            end = o + n
        if cur:
            self.buckets.append((start, end, cur))
        for bi, (_, _, ps) in enumerate(self.buckets):
            for p in ps:
                self._bucket_of[p] = bi
        if self.overlap:
            for p in active:
                if p not in self._hooked:
                    p.register_post_accumulate_grad_hook(self._on_grad)
                    self._hooked.add(p)

    # ------------------------------------------------------------ per step
    def zero(self):
        """Zero the flat gradient buffer, (re)attach the views and arm the buckets."""
        key = tuple(p.requires_grad for p in self.params)
        if key != self._active_key:
            self._layout()
            self._active_key = key
        self.flat.zero_()
        for p in self.params:
            if not p.requires_grad:
                p.grad = None
                continue
            o, n = self.views[p]
            if p.grad is None or p.grad.data_ptr() != self.flat.data_ptr() + 4 * o:
                p.grad = self.flat[o:o + n].view_as(p)
        self._left = [len(ps) for _, _, ps in self.buckets]
        self._done = set()
        self._pending = []
        if self.proxy is not None:   # a ring of 64 steps x (buckets + 1) x {ready, first start, last start, end}
            nb = len(self.buckets)
            if getattr(self, "_prx_rec", None) is None or self._prx_rec.shape[1] != nb + 1:
                self._prx_rec = torch.zeros(64, nb + 1, 4, dtype=torch.int64, device=self.flat.device)
                self._prx_step = -1
            self._prx_step += 1
            r = self._prx_rec[self._prx_step % 64]
            r.zero_()
            r[:, 1] = -1   # (UINT64_MAX: atomicMin target)

    def _is_view(self, p):
        o, _ = self.views[p]
        g = p.grad
        return g is not None and g.data_ptr() == self.flat.data_ptr() + 4 * o and g.shape == p.shape

    def grad_view(self, p):
        """``p.grad`` as this sink's flat view, for a producer that accumulates into it (the xcp
        engine's gradient sink).  After ``optimizer.zero_grad()`` (set_to_none, the reference's
        per-step call, train_visual.py:566) ``p.grad`` is None: the view is zeroed and re-attached.
        A gradient tensor of the caller's own is copied into the view first.  A parameter this
        sink does not hold keeps (or gets a zeroed) gradient tensor of its own."""
        if p not in self.views:
            if p.grad is None:
                p.grad = torch.zeros_like(p)
            return p.grad
        if not self._is_view(p):
            self._adopt(p)
        return p.grad

    def _adopt(self, p):
        o, n = self.views[p]
        v = self.flat[o:o + n].view_as(p)
        if p.grad is None:
            v.zero_()
        else:
            v.copy_(p.grad)
        p.grad = v

    def _prx_rec_row(self, i):
        return self._prx_rec[self._prx_step % 64, i]

    def _launch(self, bi):
        a, b, ps = self.buckets[bi]
        for p in ps:   # a gradient autograd created after zero_grad(set_to_none) joins the flat buffer
            if not self._is_view(p):
                self._adopt(p)
        if self.proxy is not None:
            from xcp import _lib, ops
            G = self.proxy.get("world", 8)
            bus = 2.0 * (G - 1) / G * 4 * (b - a)
            ticks = int(bus / (self.proxy.get("busbw", 300.0) * 1e9) * 1e8)
            row = self._prx_rec_row(bi)
            n16 = 4 * (b - a) // 16
            _lib.call("xcp_comm_proxy", self.flat.data_ptr() + 4 * a, self._prx_scratch.data_ptr() + 4 * a, n16,
                      int(self.proxy.get("blocks", 32)), ticks, row.data_ptr() + 8, ops.stream())
            ev = torch.cuda.Event()
            ev.record()
            self._pending.append(ev)
            return
        op = dist.ReduceOp.AVG if self.avg else dist.ReduceOp.SUM
        self._pending.append(dist.all_reduce(self.flat[a:b], op=op, async_op=True))

    def comm_stream(self):
        """The stream the bucket all-reduces are launched from (created on first use)."""
        if self._comm is None:
            self._comm = torch.cuda.Stream(self.flat.device)
        return self._comm

    def _launch_from_comm(self, bis, side_stream=None):
        """All-reduce buckets ``bis`` once the work enqueued so far on the current stream (and on
        ``side_stream``) is done, without making the current stream wait for anything."""
        if not bis:
            return
        if not self.use_streams:
            for bi in bis:   # CPU tensors (gloo): no streams
                self._launch(bi)
            return
        cur = torch.cuda.current_stream(self.flat.device)
        if DDP_LAUNCH == "main" or (DDP_LAUNCH == "side" and side_stream is None):
            if side_stream is not None:
                cur.wait_stream(side_stream)
            for bi in bis:
                self._launch(bi)
            return
        if DDP_LAUNCH == "side":
            side_stream.wait_stream(cur)
            with torch.cuda.stream(side_stream):
                for bi in bis:
                    self._launch(bi)
            return
        comm = self.comm_stream()
        comm.wait_stream(cur)
        if side_stream is not None:
            comm.wait_stream(side_stream)
        with torch.cuda.stream(comm):
            for bi in bis:
                self._launch(bi)

    def ready(self, params, side_stream=None):
        """Gradients of ``params`` are final (enqueued on the current stream, weight gradients
        possibly on ``side_stream``).  Launches the all-reduce of every bucket this completes."""
        if not self.overlap or not self.sync:
            return
        full = []
        for p in params:
            if p in self._done or p not in self._bucket_of:
                continue
            self._done.add(p)
            bi = self._bucket_of[p]
            self._left[bi] -= 1
            if self._left[bi] == 0:
                full.append(bi)
        if self.proxy is not None and full:
            from xcp import _lib, ops
            for bi in full:   # the ready point, on the current (main) stream
                _lib.call("xcp_stamp", self._prx_rec_row(bi).data_ptr(), ops.stream())
        self._launch_from_comm(full, side_stream)

    def _on_grad(self, p):
        self.ready([p])

    def allreduce(self):
        """Finish the gradient mean across ranks (no-op at world size 1).  Buckets that did not
        complete during backward (parameters without a gradient this step) are reduced here."""
        if self.proxy is not None:
            from xcp import _lib, ops
            _lib.call("xcp_stamp", self._prx_rec_row(len(self.buckets)).data_ptr(), ops.stream())   # backward end
            rest = [bi for bi in range(len(self.buckets)) if self._left[bi] != 0]
            for bi in rest:
                self._left[bi] = 0
            self._launch_from_comm(rest)
            cur = torch.cuda.current_stream(self.flat.device)
            for ev in self._pending:   # (as w.wait() on a collective)
                cur.wait_event(ev)
            self._pending = []
            return
        if self.world <= 1:
            return
        rest = []
        for bi in range(len(self.buckets)):
            if self._left[bi] != 0:
                self._left[bi] = 0
                rest.append(bi)
        self._launch_from_comm(rest)
        for w in self._pending:   # the current (main) stream waits for the collectives
            w.wait()
        self._pending = []
        if not self.avg:
            for a, b, _ in self.buckets:
                self.flat[a:b].mul_(1.0 / self.world)


def proxy_report(buckets, steps):
    """Per-bucket timings of the last ``steps`` steps of a proxy-mode GradBuckets (synchronises), in
    microseconds: ready -> first stand-in workgroup start ("start_delay"), first -> last workgroup
    start ("cu_wait"), stand-in duration, and the backward end -> last stand-in end ("exposed")."""
    import torch as _t
    _t.cuda.synchronize()
    n = min(steps, 64, buckets._prx_step + 1)
    rows = [buckets._prx_rec[(buckets._prx_step - i) % 64].cpu() for i in range(n)]
    nb = len(buckets.buckets)
    us = lambda t: t / 100.0   # noqa: E731  (100 MHz ticks)
    per = []
    for bi in range(nb):
        a, b, _ = buckets.buckets[bi]
        rd = [float(us(r[bi, 1] - r[bi, 0])) for r in rows]
        cw = [float(us(r[bi, 2] - r[bi, 1])) for r in rows]
        du = [float(us(r[bi, 3] - r[bi, 1])) for r in rows]
        per.append({"bucket_mb": round(4 * (b - a) / 1e6, 2), "start_delay_us": round(sum(rd) / n, 1),
                    "start_delay_max_us": round(max(rd), 1), "cu_wait_us": round(sum(cw) / n, 1),
                    "duration_us": round(sum(du) / n, 1)})
    exp = [float(us(max(int(r[bi, 3]) for bi in range(nb)) - r[nb, 0])) for r in rows]
    first = [float(us(min(int(r[bi, 1]) for bi in range(nb)) - r[nb, 0])) for r in rows]
    return {"steps": n, "world": buckets.proxy.get("world", 8), "busbw_gbs": buckets.proxy.get("busbw", 300.0),
            "blocks": buckets.proxy.get("blocks", 32), "buckets": per,
            "first_start_vs_backward_end_us": round(sum(first) / n, 1),
            "exposed_after_backward_us": round(sum(exp) / n, 1), "exposed_max_us": round(max(exp), 1)}


def _backbones(module):
    """the xcp Xception backbones inside ``module`` (modules carrying the buffer-wait slot)"""
    return [m for m in module.modules() if hasattr(m, "_xcp_wait_buffers")]


_BCAST = weakref.WeakKeyDictionary()   # module -> its persistent broadcast buffer and stream


def broadcast_buffers(module, src=0, use_streams=None):
    """DDP ``broadcast_buffers``: every floating-point buffer of ``module`` takes rank 0's value.

    On the GPU, when every such buffer belongs to an xcp Xception backbone, the gather, broadcast
    and scatter run on a stream of their own and the backbones' forward makes the main stream wait
    for them only at its first running-statistic access (``Xception._xcp_wait_buffers``); the
    step's first kernels are not held up.  Otherwise (CPU / gloo, or buffers outside a backbone)
    it completes on the current stream as before."""
    if not (dist.is_initialized() and dist.get_world_size() > 1):
        return
    bufs = [b for b in module.buffers() if b.is_floating_point()]
    if not bufs:
        return
    if use_streams is None:
        # RCCL enqueues the broadcast on the side stream; gloo blocks the host in wait() until the side
        # stream (which waits on the main stream) has drained, so the stream buys nothing there
        # (XCP_BCAST_STREAMS=0/1 overrides, A/B)
        env = os.environ.get("XCP_BCAST_STREAMS")
        use_streams = bufs[0].is_cuda and (env == "1" if env in ("0", "1") else dist.get_backend() == "nccl")
    bbs = _backbones(module)
    if len({(b.dtype, b.device) for b in bufs}) > 1:
        # mixed dtypes / devices (e.g. a float64 running stat): one flat buffer per group, on the
        # current stream
        for m in bbs:
            m._xcp_wait_buffers()
        groups = {}
        for b in bufs:
            groups.setdefault((b.dtype, b.device), []).append(b)
        for g in groups.values():
            flat = torch.cat([b.reshape(-1) for b in g])
            dist.broadcast(flat, src)
            torch._foreach_copy_(g, [v.view_as(b) for v, b in zip(flat.split([b.numel() for b in g]), g)])
        return
    st = _BCAST.get(module)
    n = sum(b.numel() for b in bufs)
    key = (n, bufs[0].device, bufs[0].dtype)
    if st is None or st["key"] != key:
        st = {"flat": torch.empty(n, device=bufs[0].device, dtype=bufs[0].dtype), "stream": None, "key": key}
        _BCAST[module] = st
    flat = st["flat"]
    views = [v.view_as(b) for v, b in zip(flat.split([b.numel() for b in bufs]), bufs)]
    owned = {id(b) for m in bbs for b in m.buffers() if b.is_floating_point()}
    if not (use_streams and bbs and all(id(b) in owned for b in bufs)):
        for m in bbs:
            m._xcp_wait_buffers()
        torch.cat([b.reshape(-1) for b in bufs], out=flat)
        dist.broadcast(flat, src)
        # one multi-tensor launch instead of a copy kernel per BN buffer (~80 per step)
        torch._foreach_copy_(bufs, views)
        return
    for m in bbs:   # a previous broadcast nobody waited for is complete before this one reuses flat
        m._xcp_wait_buffers()
    if st["stream"] is None:
        st["stream"] = torch.cuda.Stream(flat.device)
    side, cur = st["stream"], torch.cuda.current_stream(flat.device)
    torch.cat([b.reshape(-1) for b in bufs], out=flat)   # on the current stream: the buffers as of now
    side.wait_stream(cur)
    with torch.cuda.stream(side):
        w = dist.broadcast(flat, src, async_op=True)
        if w is not None:
            w.wait()
        torch._foreach_copy_(bufs, views)
        ev = torch.cuda.Event()
        ev.record(side)
    for m in bbs:
        m._xcp_buffer_wait = ev


def wait_buffers(module):
    """Make the current stream wait for a ``broadcast_buffers`` still in flight on ``module``'s
    backbones.  The forward, ``state_dict()``, pickling / deepcopy and nn.DataParallel replication
    of an xcp Xception do this themselves; call it before touching the BN buffers any other way
    (e.g. an in-place EMA of the running statistics outside forward)."""
    for m in _backbones(module):
        m._xcp_wait_buffers()
