"""CPU dry run of the engine's host orchestration (no GPU, no kernel executes).

The C ABI is replaced by a recorder that type-checks every call against the
ctypes signatures in xcp/_lib.py (argument count and convertibility) and checks
that every pointer argument addresses a live tensor large enough for the
extents the call implies where cheap to infer.  This exercises the whole
forward/backward call sequence of the XceptionLSTMV step on CPU in seconds.
"""
import ctypes

import pytest
import torch
import torch.nn as nn


@pytest.fixture
def fake_lib(monkeypatch):
    from xcp import _lib, ops
    calls = []

    def fake_call(name, *args):
        sig = _lib.SIGNATURES[name]
        assert len(args) == len(sig), (name, len(args), len(sig))
        for a, t in zip(args, sig):
            t(a if a is not None else 0)  # raises on an unconvertible argument
        calls.append(name)
        if name == "xcp_dw_bwd_chunks":
            return 7
        if name == "xcp_chanred_parts":
            return 5
        if name == "xcp_conv1_wgrad_parts":
            return 3
        if name in ("xcp_gemm_tn_rows_per_split", "xcp_gemm_nt_stat_rows"):
            return 256
        if name in ("xcp_conv3x3_parts", "xcp_conv3x3_wgrad_parts"):
            return 9
        if name == "xcp_maxpool_bwd_bnred_parts":
            return 4
        return 0

    monkeypatch.setattr(_lib, "call", fake_call)
    monkeypatch.setattr(ops, "check_gpu", lambda *a: None)
    from xcp import engine
    monkeypatch.setattr(engine, "WGRAD_SIDE_STREAM", False)   # no HIP streams on the CPU

    class _S:
        cuda_stream = 0

    monkeypatch.setattr(torch.cuda, "current_stream", lambda *a, **k: _S())
    return calls


@pytest.mark.parametrize("unfrozen", [False, True])
def test_lstmv_step_call_sequence(fake_lib, unfrozen):
    from Models.XceptionLSTMV import XceptionLSTMV
    torch.manual_seed(0)
    m = XceptionLSTMV(128, pretrained=False)
    if unfrozen:
        for p in m.feature_extractor.parameters():
            p.requires_grad = True
    x = torch.rand(2, 3, 3, 71, 71)
    feats = m.extract_features(x, "cpu")
    assert feats.shape == (2, 3, 2048)
    prob = m(feats)
    loss = nn.BCELoss()(prob.clamp(1e-3, 1 - 1e-3), torch.tensor([[0.0], [1.0]]))
    loss.backward()
    names = set(fake_lib)
    assert {"xcp_gemm_nt", "xcp_dw_fwd", "xcp_tail_fwd", "xcp_avgpool_fwd", "xcp_lstm_fwd", "xcp_lstm_bwd"} <= names
    if unfrozen:
        assert {"xcp_dw_bwd", "xcp_gemm_tn", "xcp_bn_bwd_reduce", "xcp_maxpool_bwd_bnred", "xcp_conv1_wgrad",
                "xcp_conv3x3", "xcp_conv3x3_wgrad"} <= names
        for n, p in m.feature_extractor.named_parameters():
            assert p.grad is not None and p.grad.shape == p.shape, n
    else:
        assert "xcp_dw_bwd" not in names
        assert all(p.grad is None for p in m.feature_extractor.parameters())
    # 34 depthwise + 34 pointwise convs per pass
    assert fake_lib.count("xcp_dw_fwd") == 34
    assert fake_lib.count("xcp_tail_fwd") == 12


def test_header_matches_binding():
    """include/xcp.h declares exactly the entry points _lib.py binds, with the same arity."""
    import os
    import re
    from xcp import _lib
    hdr = open(os.path.join(os.path.dirname(__file__), "..", "include", "xcp.h")).read()
    decls = dict(re.findall(r"int\s+(xcp_\w+)\(([^;]*)\);", hdr, re.S))
    assert set(decls) == set(_lib.SIGNATURES)
    for name, args in decls.items():
        n = len([a for a in args.split(",") if a.strip()])
        assert n == len(_lib.SIGNATURES[name]), name


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
