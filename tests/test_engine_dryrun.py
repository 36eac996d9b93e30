"""CPU dry run of the engine's host orchestration (no GPU, no kernel executes).

The C ABI is replaced by a recorder that type-checks every call against the
ctypes signatures in xcp/_lib.py (argument count and convertibility) and checks
that every pointer argument addresses a live tensor large enough for the
extents the call implies where cheap to infer.  This exercises the whole
forward/backward call sequence of the XceptionLSTMV step on CPU in seconds.
"""
import contextlib
import ctypes
import os

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp
import torch.nn as nn

# value the fake kernels write into every gradient they produce (rank-dependent under gloo)
FILL = {"v": 1.0}


def _fill(ptr, n, acc):
    """write (acc: add) FILL into n fp32 elements at a host address (dry-run tensors are CPU)"""
    a = (ctypes.c_float * n).from_address(ptr)
    for i in range(n):
        a[i] = (a[i] if acc else 0.0) + FILL["v"]


def install_fake_lib(monkeypatch):
    from xcp import _lib, ops
    calls = []

    def fake_call(name, *args):
        sig = _lib.SIGNATURES[name]
        assert len(args) == len(sig), (name, len(args), len(sig))
        for a, t in zip(args, sig):
            t(a if a is not None else 0)  # raises on an unconvertible argument
        calls.append(name)
        if name == "xcp_colreduce_f32":       # (in, S, L, ld, out, G, accumulate, stream): gradient slabs
            _fill(args[4], args[2] * args[5], args[6])
        elif name == "xcp_colreduce_multi":   # (jobs [n][7] = in, out, S, L, ld, G, acc; n; stream)
            jobs = (ctypes.c_longlong * (7 * args[1])).from_address(args[0])
            for i in range(args[1]):
                _, out, _, L, _, G, acc = jobs[7 * i:7 * i + 7]
                _fill(out, L * G, acc)
        elif name == "xcp_bn_bwd_finalize_part" and args[11]:   # dgamma, dbeta (C each)
            _fill(args[11], args[2], args[13] & 1)   # (flags: 1 accumulate, 2 narrow)
            _fill(args[12], args[2], args[13] & 1)
        elif name == "xcp_permute3" and args[0] == 0:          # fp32 permute (stem conv2 gradient)
            _fill(args[2], args[3] * args[4] * args[5], False)
        if name == "xcp_dw_bwd_chunks":
            return 7
        if name == "xcp_chanred_parts":
            return 5
        if name == "xcp_conv1_wgrad_parts":
            return 3
        if name == "xcp_conv1_fwd_parts":
            return 3
        if name == "xcp_conv1_wgrad_fused":   # (dtype, IH, IW): the row kernel takes bf16 frames <= 320 wide
            return 1 if args[0] == 1 and args[2] <= 320 else 0
        if name in ("xcp_gemm_tn_rows_per_split", "xcp_gemm_nt_stat_rows"):
            return 256
        if name in ("xcp_conv3x3_parts", "xcp_conv3x3_wgrad_parts"):
            return 9
        if name == "xcp_maxpool_bwd_bnred_parts":
            return 4
        if name == "xcp_sep_fwd_parts":   # (dtype, N, H, W, CIN, COUT): block1's fused forward
            ok = args[0] == 1 and ((args[4] in (64, 128) and args[5] == 128 and args[3] <= 152) or
                                   (args[4] == 128 and args[5] == 256 and args[3] <= 78))
            return min(args[1], 256) if ok else 0
        if name == "xcp_unit_bwd_rows_per_split":   # (dtype, M, CO, CI): the fused narrow unit
            ok = args[0] == 1 and (args[2], args[3]) in ((128, 64), (128, 128), (256, 128), (256, 256))
            return 64 if ok else 0
        return 0

    monkeypatch.setattr(_lib, "call", fake_call)
    monkeypatch.setattr(ops, "check_gpu", lambda *a: None)
    monkeypatch.setattr(ops, "device_guard", lambda t: contextlib.nullcontext())
    from xcp import engine
    monkeypatch.setattr(engine, "WGRAD_SIDE_STREAM", False)   # no HIP streams on the CPU

    class _S:
        cuda_stream = 0

    monkeypatch.setattr(torch.cuda, "current_stream", lambda *a, **k: _S())

    # the LSTM custom op is registered for the GPU only: drive its Python bodies directly
    from xcp import lstm as xl, torch_ops as T

    class _LSTMFn(torch.autograd.Function):
        @staticmethod
        def forward(ctx, x, w_ih, w_hh, b_ih, b_hh):
            out, hn, cn, hprev, cst, gates = T.lstm._init_fn(x, w_ih, w_hh, b_ih, b_hh, 0)
            ctx.save_for_backward(x, w_ih, w_hh, hprev, cst, gates)
            return out, hn, cn

        @staticmethod
        def backward(ctx, dout, dhn, dcn):
            x, w_ih, w_hh, hprev, cst, gates = ctx.saved_tensors
            dx, dw_ih, dw_hh, db = T.lstm_backward._init_fn(dout, dhn, dcn, x, w_ih, w_hh, hprev, cst, gates, 0, False)
            return None, dw_ih, dw_hh, db, db.clone()

    def fake_forward(self, input, hx=None):
        out, hn, cn = _LSTMFn.apply(input, self.weight_ih_l0, self.weight_hh_l0, self.bias_ih_l0, self.bias_hh_l0)
        return out, (hn, cn)

    monkeypatch.setattr(xl.LSTM, "forward", fake_forward)
    return calls


@pytest.fixture
def fake_lib(monkeypatch):
    return install_fake_lib(monkeypatch)


@pytest.mark.parametrize("prec", ["bf16", "fp32"])
@pytest.mark.parametrize("unfrozen", [False, True])
@pytest.mark.parametrize("resbn", [False, True])
def test_lstmv_step_call_sequence(fake_lib, monkeypatch, unfrozen, prec, resbn):
    import xcp
    from xcp import engine as engine_mod
    from Models.XceptionLSTMV import XceptionLSTMV
    monkeypatch.setattr(engine_mod, "RESBN", resbn)
    # (71^2 frames: block1 at 33^2, narrower than the fused forward's default minimum; the call
    # sequence is checked with it on, test_sep_fwd_width_gate checks the default)
    monkeypatch.setattr(engine_mod, "SEP_MIN_W", {128: 0, 256: 0})
    torch.manual_seed(0)
    m = XceptionLSTMV(128, pretrained=False)
    if unfrozen:
        for p in m.feature_extractor.parameters():
            p.requires_grad = True
    x = torch.rand(2, 3, 3, 71, 71)
    with xcp.precision(prec):
        feats = m.extract_features(x, "cpu")
        assert feats.shape == (2, 3, 2048)
        prob = m(feats)
        loss = torch.nan_to_num(prob).sum()   # (the fake kernels leave their outputs uninitialised)
        loss.backward()
    names = set(fake_lib)
    assert {"xcp_gemm_nt", "xcp_dw_fwd", "xcp_tail_fwd", "xcp_avgpool_fwd", "xcp_lstm_fwd", "xcp_lstm_bwd"} <= names
    if unfrozen:
        assert {"xcp_dw_bwd", "xcp_gemm_tn", "xcp_bn_bwd_reduce", "xcp_maxpool_bwd_bnred"} <= names
        # conv1's weight gradient: BN1's backward apply fused into it in bf16, apply + plain form in fp32
        assert ("xcp_conv1_wgrad_bn" in names) == (prec == "bf16")
        assert ("xcp_conv1_wgrad" in names) == (prec == "fp32")
        # stem conv2: direct MFMA conv in bf16, im2col GEMM (gather modes 2 / 3) in fp32
        assert ({"xcp_conv3x3", "xcp_conv3x3_wgrad"} <= names) == (prec == "bf16")
        # block1's and block2's units (64/128 -> 128, 128/256 -> 256): fused BN-apply + pointwise
        # dgrad + wgrad in bf16
        assert fake_lib.count("xcp_unit_bwd") == (4 if prec == "bf16" else 0)
        # identity-skip boundaries (blocks 5-11 after an unpooled block): the previous block's last BN
        # sums come from the first depthwise backward, not from a per-channel reduce
        assert fake_lib.count("xcp_dw_bwd_resbn") == (7 if resbn else 0)
        for n, p in m.feature_extractor.named_parameters():
            assert p.grad is not None and p.grad.shape == p.shape, n
    else:
        assert "xcp_dw_bwd" not in names
        assert all(p.grad is None for p in m.feature_extractor.parameters())
    # 34 depthwise + 34 pointwise convs per pass; in bf16 block1's two units and block2's
    # first run depthwise + pointwise as one fused launch
    assert fake_lib.count("xcp_sep_fwd") == (3 if prec == "bf16" else 0)
    assert fake_lib.count("xcp_dw_fwd") == 34 - fake_lib.count("xcp_sep_fwd")
    assert fake_lib.count("xcp_tail_fwd") == 12


def test_sep_fwd_width_gate(fake_lib):
    """block1's / block2's fused depthwise + pointwise forward only on frames wide enough for its
    80-pixel half rows (engine.SEP_MIN_W): 71^2 clips (block1 at 33^2, block2 at 17^2) take the two
    kernels, bitwise the same results (test_sep_fwd_vs_dw_and_gemm)"""
    import xcp
    from xcp import engine as engine_mod
    from Models.XceptionLSTMV import XceptionLSTMV
    assert engine_mod.SEP_MIN_W == {128: 120, 256: 64}
    torch.manual_seed(0)
    m = XceptionLSTMV(128, pretrained=False)
    with xcp.precision("bf16"):
        feats = m.extract_features(torch.rand(2, 3, 3, 71, 71), "cpu")
        torch.nan_to_num(m(feats)).sum().backward()
    assert fake_lib.count("xcp_sep_fwd") == 0
    assert fake_lib.count("xcp_dw_fwd") == 34


def test_weights_repacked_after_fused_optimizer_step(fake_lib):
    """FusedAdamClip writes the parameters through raw pointers; it bumps their version counters,
    so the next forward repacks the kernel-layout weights (one batched permute launch per
    direction) instead of running on the pre-step copies."""
    from xcp import ops, optim
    from Models.Xception import xception
    ops_check = ops.check_gpu
    try:
        ops.check_gpu = lambda *a: None   # (the optimiser checks its parameters at construction)
        torch.manual_seed(0)
        m = xception(num_classes=1)
        opt = optim.FusedAdamClip(m.parameters(), lr=1e-3, max_norm=1.0)
    finally:
        ops.check_gpu = ops_check
    packs = []
    for _ in range(3):
        n0 = len(fake_lib)
        m(torch.rand(2, 3, 71, 71)).sum().backward()
        packs.append(fake_lib[n0:].count("xcp_permute3_batch"))
        v0 = m.conv1.weight._version
        opt.step()
        assert m.conv1.weight._version == v0 + 1
        opt.zero_grad()
    assert packs == [2, 2, 2], packs   # forward + backward layouts, every step


def test_header_matches_binding():
    """include/xcp.h declares exactly the entry points _lib.py binds, with the same arity."""
    import os
    import re
    from xcp import _lib
    hdr = open(os.path.join(os.path.dirname(__file__), "..", "include", "xcp.h")).read()
    decls = dict(re.findall(r"int\s+(xcp_\w+)\(([^;]*)\);", hdr, re.S))
    assert set(decls) == set(_lib.SIGNATURES)
    for name, args in decls.items():
        n = len([a for a in args.split(",") if a.strip() and a.strip() != "void"])
        assert n == len(_lib.SIGNATURES[name]), name


def test_header_constants_match_kernel_enums():
    """Every XCP_* constant the C header defines that the kernels' common.h also defines (dtypes, statuses,
    the finalize flags) has the same value on both sides of the ABI."""
    import os
    import re
    root = os.path.join(os.path.dirname(__file__), "..")
    hdr = open(os.path.join(root, "include", "xcp.h")).read()
    common = open(os.path.join(root, "multimodal-deepfake-detection_amd", "xcp", "csrc", "common.h")).read()
    h = {k: int(v) for k, v in re.findall(r"#define\s+(XCP_[A-Z0-9_]+)\s+(-?\d+)\b", hdr)}
    c = {k: int(v) for k, v in re.findall(r"\b(XCP_[A-Z0-9_]+)\s*=\s*(-?\d+)", common)}
    shared = set(h) & set(c)
    assert {"XCP_OK", "XCP_EINVAL", "XCP_EUNSUPPORTED", "XCP_F32", "XCP_BF16", "XCP_FIN_ACCUMULATE",
            "XCP_FIN_NARROW"} <= shared, sorted(shared)
    for k in shared:
        assert h[k] == c[k], k


def test_library_exports_every_symbol():
    """libxcp.so (built in-tree) loads and exports every symbol of include/xcp.h.
    Loading needs no GPU; no compute call is made."""
    from xcp import _lib
    import os
    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("libxcp.so not built (run __graft_entry__.build())")
    lib = ctypes.CDLL(_lib.LIB_PATH)
    for name in _lib.SIGNATURES:
        assert hasattr(lib, name), name


def test_no_cpu_fallback():
    from Models.Xception import xception
    m = xception(num_classes=1)
    with pytest.raises(RuntimeError, match="MI355X"):
        m(torch.zeros(1, 3, 64, 64))


def test_default_mode_returns_gradients_to_autograd(fake_lib):
    """Without a gradient sink the backbone node hands its gradients to autograd:
    torch.autograd.grad works and post-accumulate-grad hooks fire for backbone parameters."""
    from Models.Xception import xception
    torch.manual_seed(0)
    m = xception(num_classes=1)
    m.fc = nn.Identity()
    params = list(m.parameters())
    fired = []
    for p in params:
        p.register_post_accumulate_grad_hook(lambda p: fired.append(p))
    f = m(torch.rand(2, 3, 71, 71))
    gr = torch.autograd.grad(f.sum(), [m.block4.rep[1].pointwise.weight, m.conv1.weight])
    assert all(g is not None and torch.all(g == FILL["v"]) for g in gr)
    assert m.block4.rep[1].pointwise.weight.grad is None      # autograd.grad leaves .grad alone
    m(torch.rand(2, 3, 71, 71)).sum().backward()
    assert len(fired) == len(params)


def _sink_worker(rank, world, port, out):
    """gloo rank: the engine's hook-less accumulation path with GradBuckets as its sink."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)

    class _MP:   # minimal monkeypatch for a spawned process
        def setattr(self, obj, name, val):
            setattr(obj, name, val)

    calls = install_fake_lib(_MP())
    FILL["v"] = float(rank + 1)
    from xcp import ddp
    from Models.Xception import xception
    torch.manual_seed(0)
    m = xception(num_classes=1)
    m.fc = nn.Identity()
    params = list(m.parameters())
    events = []
    real = ddp.dist.all_reduce

    def logged(t, *a, **k):
        events.append(len(calls))
        return real(t, *a, **k)

    ddp.dist.all_reduce = logged
    gb = ddp.GradBuckets(params, bucket_bytes=1 << 20, world=world, module=m)
    for step in range(2):
        gb.zero()
        if step == 1:   # optimizer.zero_grad() (set_to_none) after zero(): the sink re-attaches its views
            for p in params:
                p.grad = None
        events.clear()
        n0 = len(calls)
        m(torch.rand(2, 3, 71, 71)).sum().backward()
        last_dw = max(i for i, c in enumerate(calls) if c == "xcp_dw_bwd")
        launched_during = sum(1 for e in events if e <= last_dw)
        gb.allreduce()
    out[rank] = {"grads": {n: p.grad.clone() for n, p in m.named_parameters()}, "during": launched_during,
                 "buckets": len(gb.buckets), "nbwd": len(calls) - n0}
    dist.destroy_process_group()


def test_sink_allreduce_overlaps_backbone_backward():
    """world 2 (gloo), fake kernels writing rank+1 into every gradient: the engine accumulates
    into GradBuckets' views, buckets are all-reduced while the backbone backward is still
    being enqueued, and every backbone gradient ends as the mean over ranks (1.5)."""
    world, port = 2, 29600 + os.getpid() % 1000
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_sink_worker, args=(world, port, out), nprocs=world, join=True)
    for rank in range(world):
        r = out[rank]
        assert r["buckets"] > 4
        assert r["during"] >= r["buckets"] - 2, r   # all but the stem buckets launched inside backward
        for n, gr in r["grads"].items():
            assert torch.all(gr == 1.5), n


class _FakeStream:
    """A recording stand-in for torch.cuda.Stream on the CPU: wait_stream logs
    (waiter, waited-on, number of library calls enqueued so far)."""
    log, calls, current, n = [], None, None, 0

    def __init__(self, device=None, priority=0, name=None):
        _FakeStream.n += 1
        self.device, self.name, self.cuda_stream = device, name or f"s{_FakeStream.n}", 0

    def wait_stream(self, other):
        _FakeStream.log.append((self.name, other.name, len(_FakeStream.calls)))

    def wait_event(self, ev):
        _FakeStream.log.append((self.name, ev.stream.name, len(_FakeStream.calls)))


class _FakeEvent:
    def __init__(self, *a, **k):
        self.stream = None

    def record(self, stream=None):
        self.stream = stream or _FakeStream.current


def _install_fake_streams(calls):
    _FakeStream.log, _FakeStream.calls = [], calls
    _FakeStream.current = _FakeStream(name="main")

    @contextlib.contextmanager
    def stream(s):
        prev, _FakeStream.current = _FakeStream.current, s
        try:
            yield
        finally:
            _FakeStream.current = prev

    torch.cuda.Stream = _FakeStream
    torch.cuda.Event = _FakeEvent
    torch.cuda.stream = stream
    torch.cuda.current_stream = lambda *a, **k: _FakeStream.current


def _streams_worker(rank, world, port, out):
    """gloo rank: the engine with its weight-gradient side stream (recording fake streams) and
    GradBuckets launching bucket all-reduces from its communication stream."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)

    class _MP:
        def setattr(self, obj, name, val):
            setattr(obj, name, val)

    calls = install_fake_lib(_MP())
    FILL["v"] = float(rank + 1)
    from xcp import ddp, engine
    engine.WGRAD_SIDE_STREAM = True
    _install_fake_streams(calls)
    from Models.Xception import xception
    torch.manual_seed(0)
    m = xception(num_classes=1)
    m.fc = nn.Identity()
    params = list(m.parameters())
    launched = []
    real = ddp.dist.all_reduce

    def logged(t, *a, **k):
        launched.append((len(calls), _FakeStream.current.name))
        return real(t, *a, **k)

    ddp.dist.all_reduce = logged
    gb = ddp.GradBuckets(params, bucket_bytes=1 << 20, world=world, module=m)
    gb.use_streams = True
    gb.zero()
    with torch.no_grad():   # rank-dependent buffers: the broadcast must leave rank 0's everywhere
        for b in m.buffers():
            if b.is_floating_point():
                b.fill_(rank + 1.0)
    n_bc = len(calls)
    ddp.broadcast_buffers(m, use_streams=True)
    bstream = ddp._BCAST[m]["stream"].name
    m(torch.rand(2, 3, 71, 71)).sum().backward()
    last_dw = max(i for i, c in enumerate(calls) if c == "xcp_dw_bwd")
    first_fin = min(i for i, c in enumerate(calls) if c.startswith("xcp_bn_finalize"))
    gb.allreduce()
    side = m._engine()._side.name
    out[rank] = {"log": list(_FakeStream.log), "launched": launched, "last_dw": last_dw, "side": side,
                 "buckets": len(gb.buckets), "grads_ok": all(torch.all(p.grad == 1.5).item() for p in params),
                 "bstream": bstream, "n_bc": n_bc, "first_fin": first_fin, "bufs_ok": all(
                     torch.all(b == 1.0).item() for b in m.buffers() if b.is_floating_point()),
                 "avg": gb.avg}
    dist.destroy_process_group()


def test_bucket_allreduce_does_not_stall_main_stream():
    """world 2 (gloo), fake kernels, recording fake streams: every bucket
    all-reduce completed during the backbone backward is launched from the engine's
    weight-gradient side stream after that stream waits on the main stream; the main stream is
    never made to wait on the side stream before the backbone backward has been enqueued (only
    the engine's own wait at its end), and every backbone gradient is the mean over ranks."""
    world, port = 2, 29700 + os.getpid() % 1000
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_streams_worker, args=(world, port, out), nprocs=world, join=True)
    for rank in range(world):
        r = out[rank]
        assert r["grads_ok"]
        during = [(n, st) for n, st in r["launched"] if n <= r["last_dw"]]
        assert len(during) >= r["buckets"] - 2, r
        assert all(st == r["side"] for _, st in during), during
        main_waits_side = [n for w, o, n in r["log"] if w == "main" and o == r["side"]]
        assert all(n > r["last_dw"] for n in main_waits_side), (main_waits_side, r["last_dw"])
        # before each launch from the side stream, the side stream waited on the main stream
        side_waits_main = [n for w, o, n in r["log"] if w == r["side"] and o == "main"]
        assert all(any(m <= n for m in side_waits_main) for n, _ in during)
        # broadcast_buffers: launched from a stream of its own after it waits on
        # the main stream; the main stream waits for it once, after the forward's first kernel
        # (conv1) and at the first running-statistic access (BN1's finalize), not at step start
        assert r["bufs_ok"] and r["bstream"] not in ("main", r["side"])
        assert (r["bstream"], "main", r["n_bc"]) in r["log"]
        main_waits_b = [n for w, o, n in r["log"] if w == "main" and o == r["bstream"]]
        assert len(main_waits_b) == 1 and r["n_bc"] < main_waits_b[0] <= r["first_fin"], (main_waits_b, r)
        assert not r["avg"]   # gloo has no ReduceOp.AVG: SUM and one scaling pass


def _cpu_replicate(net):
    """torch.nn.parallel.replicate for one replica, on the CPU (the real one broadcasts over
    CUDA devices): every module through _replicate_for_data_parallel, parameters as non-leaf
    copies set as plain attributes (and in _former_parameters), buffers cloned."""
    from collections import OrderedDict
    modules = list(net.modules())
    idx = {m: i for i, m in enumerate(modules)}
    copies = [m._replicate_for_data_parallel() for m in modules]
    pcopy = {p: p * 1.0 for p in net.parameters()}
    for m, r in zip(modules, copies):
        r._former_parameters = OrderedDict()
        for k, child in m._modules.items():
            if child is None:
                r._modules[k] = None
            else:
                setattr(r, k, copies[idx[child]])
        for k, p in m._parameters.items():
            if p is None:
                r._parameters[k] = None
            else:
                setattr(r, k, pcopy[p])
                r._former_parameters[k] = pcopy[p]
        for k, b in m._buffers.items():
            setattr(r, k, None if b is None else b.clone())
    return copies[0]


def test_dataparallel_replica_gets_own_engine(fake_lib):
    """nn.DataParallel (train_audio.py:16-18) replicates with a shallow __dict__ copy: a replica
    must not drive the original's engine (bound to the original's parameters on cuda:0), must
    not feed its gradient sink, and its backbone gradients must reach the original parameters
    through the broadcast copies."""
    from xcp import ddp
    from Models.Xception import xception
    torch.manual_seed(0)
    m = xception(num_classes=1)
    m.fc = nn.Identity()
    gb = ddp.GradBuckets(list(m.parameters()), module=m)
    m(torch.rand(2, 3, 71, 71))                     # the original's engine exists now
    eng0 = m._engine()
    r = _cpu_replicate(m)
    assert r._xcp_engines is not m._xcp_engines and not r._xcp_engines
    assert r._xcp_grad_sink is None and m._xcp_grad_sink is gb
    er = r._engine()
    assert er is not eng0 and er.model is r and eng0.model is m
    names0 = [n for n, _ in eng0.named_params()]
    namesr = [n for n, _ in er.named_params()]
    assert names0 == namesr and len(namesr) == len(list(m.parameters()))
    assert all(t is getattr(r.get_submodule(n.rsplit(".", 1)[0]) if "." in n else r, n.rsplit(".", 1)[-1])
               for n, t in er.named_params())
    for p in m.parameters():
        p.grad = None
    r(torch.rand(2, 3, 71, 71)).sum().backward()
    for n, p in m.named_parameters():              # through the copies, not the sink
        assert p.grad is not None and torch.all(p.grad == FILL["v"]), n
    # a plain shallow copy (no _replicate_for_data_parallel) still gets an engine of its own
    import copy as _copy
    s = _copy.copy(m)
    assert s._engine().model is s and m._engine() is eng0


def test_sink_reattaches_after_zero_grad_set_to_none(fake_lib):
    """optimizer.zero_grad() (set_to_none, the reference's per-step call, train_visual.py:566)
    between GradBuckets.zero() steps: the engine's gradient sink re-attaches the zeroed flat
    views instead of accumulating into fresh tensors the all-reduce never sees."""
    from xcp import ddp
    from Models.Xception import xception
    torch.manual_seed(0)
    m = xception(num_classes=1)
    m.fc = nn.Identity()
    params = list(m.parameters())
    gb = ddp.GradBuckets(params, world=1, module=m)
    for step in range(2):
        for p in params:
            p.grad = None                            # optimizer.zero_grad()
        m(torch.rand(2, 3, 71, 71)).sum().backward()
        for p in params:
            assert gb._is_view(p)
            assert torch.all(p.grad == FILL["v"])    # zeroed before accumulation, not stale


def test_rccl_allreduce_averages_inside_the_collective(fake_lib, monkeypatch):
    """On RCCL ("nccl" backend) the bucket all-reduces use ReduceOp.AVG and no scaling pass over the
    flat buffer follows; the flat buffer is left exactly as the collective wrote
    it."""
    from xcp import ddp
    ops_seen = []

    class _W:
        def wait(self):
            pass

    def fake_all_reduce(t, op=None, async_op=False):
        ops_seen.append(op)
        t.fill_(0.25)   # what the collective wrote: must not be rescaled afterwards
        return _W()

    monkeypatch.setattr(ddp.dist, "is_initialized", lambda: True)
    monkeypatch.setattr(ddp.dist, "get_backend", lambda *a: "nccl")
    monkeypatch.setattr(ddp.dist, "all_reduce", fake_all_reduce)
    ps = [torch.zeros(1000, requires_grad=True), torch.zeros(37, requires_grad=True)]
    gb = ddp.GradBuckets(ps, bucket_bytes=2048, world=4)
    assert gb.avg
    gb.zero()
    for p in ps:
        p.grad.fill_(1.0)
    gb.allreduce()
    assert ops_seen and all(o == ddp.dist.ReduceOp.AVG for o in ops_seen)
    for p in ps:
        assert torch.all(p.grad == 0.25)
