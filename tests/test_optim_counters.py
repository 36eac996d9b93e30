"""FusedAdamClip(capturable=True) keeps torch Adam's per-parameter step counts (CPU, no kernel runs).

The device step counters are regrouped on the host by which parameters hold them; the two optimiser
entry points are replaced by a numpy restatement of csrc/optim.hip's update (the chunk table rows are
host addresses on the CPU), so the host bookkeeping is what is tested here: a parameter that gets
its first gradient at step 3 (the reference unfreezes its backbone after epoch 3,
train_visual.py:547-556), a parameter whose grad is None on some steps, and a loaded state whose count
differs from its group's -- each against torch.optim.Adam on the same gradients.
"""
import contextlib
import copy
import ctypes

import numpy as np
import pytest
import torch


def _arr(ptr, n):
    return np.ctypeslib.as_array((ctypes.c_float * n).from_address(ptr))


@pytest.fixture
def fake_opt(monkeypatch):
    from xcp import _lib, ops
    launches = []

    def fake_call(name, *args):
        if name == "xcp_opt_adam_dev":
            tab, n, coef, lr, b1, b2, eps, wd, tdev, _ = args
            rows = np.ctypeslib.as_array((ctypes.c_longlong * (6 * n)).from_address(tab)).reshape(n, 6)
            t = float(_arr(tdev, 1)[0])
            launches.append(t)
            bc1 = np.float32(1.0 - b1 ** t)
            bc2 = np.float32(np.sqrt(1.0 - b2 ** t))
            for p, g, m, v, o, L in rows:
                P, G, M, V = (_arr(int(a) + 4 * int(o), int(L)) for a in (p, g, m, v))
                gi = G + np.float32(wd) * P
                M[:] = np.float32(b1) * M + np.float32(1 - b1) * gi
                V[:] = np.float32(b2) * V + np.float32(1 - b2) * gi * gi
                P[:] = P - np.float32(lr) / bc1 * M / (np.sqrt(V) / bc2 + np.float32(eps))
            return 0
        raise AssertionError(name)

    class _S:
        cuda_stream = 0

    monkeypatch.setattr(_lib, "call", fake_call)
    monkeypatch.setattr(ops, "check_gpu", lambda *a: None)
    monkeypatch.setattr(ops, "device_guard", lambda t: contextlib.nullcontext())
    monkeypatch.setattr(torch.cuda, "current_stream", lambda *a, **k: _S())
    monkeypatch.setattr(torch.cuda, "is_current_stream_capturing", lambda: False)
    return launches


def _run(params_a, params_b, opt_a, opt_b, grads_per_step):
    for step_grads in grads_per_step:
        for pa, pb, g in zip(params_a, params_b, step_grads):
            pa.grad = None if g is None else g.clone()
            pb.grad = None if g is None else g.clone()
        opt_a.step()
        opt_b.step()


def _make(shapes, seed):
    gen = torch.Generator().manual_seed(seed)
    init = [torch.randn(s, generator=gen) for s in shapes]
    return [t.clone().requires_grad_(True) for t in init], [t.clone().requires_grad_(True) for t in init], gen


def test_late_first_gradient_gets_its_own_count(fake_opt):
    """parameter 1 gets its first gradient at step 3 and parameter 2 skips step 4: both must see bias
    corrections of their own step counts, as in torch Adam (a shared group count would make their
    first updates ~3x too large)"""
    from xcp.optim import FusedAdamClip
    shapes = [(37, 5), (64,), (3, 3, 3)]
    pa, pb, gen = _make(shapes, 3)
    ref = torch.optim.Adam(pa, lr=1e-2, weight_decay=1e-4)
    opt = FusedAdamClip(pb, lr=1e-2, weight_decay=1e-4, capturable=True)
    sched = []
    for k in range(6):
        sched.append([torch.randn(s, generator=gen) if not ((i == 1 and k < 2) or (i == 2 and k == 3)) else None
                      for i, s in enumerate(shapes)])
    _run(pa, pb, ref, opt, sched)
    for p, q in zip(pa, pb):
        torch.testing.assert_close(q, p, rtol=2e-6, atol=2e-7)
        assert float(opt.state[q]["step"]) == float(ref.state[p]["step"])
    # counts 6 / 4 / 5: three distinct counters now, and one launch per counter on the last step
    assert sorted(float(opt.state[q]["step"]) for q in pb) == [4.0, 5.0, 6.0]
    assert len(fake_opt) == 1 + 1 + 2 + 2 + 3 + 3


def test_equal_counts_share_one_launch(fake_opt):
    from xcp.optim import FusedAdamClip
    shapes = [(10,), (4, 4), (7,)]
    pa, pb, gen = _make(shapes, 4)
    ref = torch.optim.Adam(pa, lr=1e-3)
    opt = FusedAdamClip(pb, lr=1e-3, capturable=True)
    _run(pa, pb, ref, opt, [[torch.randn(s, generator=gen) for s in shapes] for _ in range(3)])
    assert fake_opt == [1.0, 2.0, 3.0]
    assert len({id(opt.state[q]["step"]) for q in pb}) == 1
    for p, q in zip(pa, pb):
        torch.testing.assert_close(q, p, rtol=2e-6, atol=2e-7)


def test_loaded_states_with_different_counts(fake_opt):
    """a state dict whose parameters hold different counts loads into separate counters instead of
    overwriting one shared counter"""
    from xcp.optim import FusedAdamClip
    shapes = [(12,), (5, 2)]
    pa, pb, gen = _make(shapes, 5)
    ref = torch.optim.Adam(pa, lr=1e-2)
    sched = [[torch.randn(shapes[0], generator=gen), None], [torch.randn(shapes[0], generator=gen),
             torch.randn(shapes[1], generator=gen)]]
    for g in sched:
        for p, gg in zip(pa, g):
            p.grad = gg
        ref.step()
    opt = FusedAdamClip(pb, lr=1e-2, capturable=True)
    with torch.no_grad():
        for p, q in zip(pa, pb):
            q.copy_(p)
    opt.load_state_dict(copy.deepcopy(ref.state_dict()))   # (load_state_dict would share the moments)
    more = [[torch.randn(s, generator=gen) for s in shapes] for _ in range(2)]
    _run(pa, pb, ref, opt, more)
    for p, q in zip(pa, pb):
        torch.testing.assert_close(q, p, rtol=2e-6, atol=2e-7)
        assert float(opt.state[q]["step"]) == float(ref.state[p]["step"])
