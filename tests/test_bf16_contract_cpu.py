"""CPU checks of the bf16 contract machinery (tests/bf16_contract.py).

* The decorrelation premise: scaling the input clip by c and conv1's weight by 1/c
  (bf16_contract.scaled_input) leaves the loss and every gradient of the reference graph
  unchanged -- fp64 to 1e-12, fp32 to its own rounding noise -- so the autocast realizations at different c are
  draws of bf16 noise around ONE answer.
* The bound arithmetic: TOL where PyTorch's bf16 is closer than TOL / K_RMS, K_RMS x the RMS of its
  realizations above that, the engine's median realization against it, the pooled noise-scale ratio
  RHO, and the assertions fire on an error beyond the bound or RHO beyond RHO_MAX.
"""
import pytest
import torch

import bf16_contract as C


def seeded(shape, seed):
    return torch.rand(shape, generator=torch.Generator().manual_seed(seed), dtype=torch.float32)


# fp32: the nearly cancelling BN affine sums carry ~1e-3 of fp32 rounding noise themselves (the
# fp32 contract's 5e-3 for them), two orders below the bf16 noise the realizations sample
@pytest.mark.parametrize("dt,lim", [(torch.float64, 1e-12), (torch.float32, 5e-3)])
def test_scaled_input_leaves_gradients_unchanged(dt, lim):
    from Models.Xception import xception
    from oracle import xception_oracle as O
    torch.manual_seed(0)
    m = xception(num_classes=1000)
    m.fc = torch.nn.Identity()
    sd = {k: (v.detach().to(dt) if v.is_floating_point() else v.clone()) for k, v in m.state_dict().items()}
    x = seeded((2, 3, 64, 64), 11).to(dt)
    r = torch.randn((2, 2048), generator=torch.Generator().manual_seed(12)).to(dt)
    grads = {}
    for c in C.SCALES[:3]:
        p = {k: (v.clone().requires_grad_(True) if v.is_floating_point() and "running" not in k else v.clone())
             for k, v in sd.items()}
        q, xc = C.scaled_input(p, x, c)
        loss = (O.backbone_forward(xc, q, True, {}) * r).sum()
        loss.backward()
        grads[c] = (loss.item(), {k: v.grad.double().norm().item() for k, v in p.items() if v.grad is not None})
    l0, g0 = grads[C.SCALES[0]]
    assert len(g0) == sum(1 for k, v in sd.items() if v.is_floating_point() and "running" not in k)
    for c in C.SCALES[1:3]:
        lc, gc = grads[c]
        assert abs(lc - l0) <= min(lim, 1e-4) * abs(l0)
        worst = max(abs(gc[k] - g0[k]) / max(g0[k], 1e-30) for k in g0)
        assert worst < lim, (c, worst)


def test_bound_and_check():
    auto = {"a": [0.001, 0.01, 0.004], "b": [0.05, 0.2, 0.1]}
    rb = (sum(v * v for v in auto["b"]) / 3) ** 0.5
    assert C.bound("a", auto) == C.TOL                      # K_RMS x rms below TOL
    assert C.bound("b", auto) == pytest.approx(C.K_RMS * rb)
    assert C.bound("c", auto) == C.TOL
    assert C.bound("a", None) == C.TOL
    assert C.med([0.3, 0.01, 0.02]) == 0.02 and C.med(0.3) == 0.3
    r, n = C.rho({"a": [0.002, 0.004, 0.006], "b": [0.1, 0.1, 0.1], "c": 0.5}, auto)
    assert n == 2 and r == pytest.approx(((0.004 / C.rms(auto["a"])) ** 2 / 2 + (0.1 / rb) ** 2 / 2) ** 0.5
                                         / C.MED3_M2 ** 0.5)
    if C.RECORD:
        pytest.skip("XCP_BF16_RECORD=1 does not assert")
    C.check("t", {"a": 0.049, "b": 0.99 * C.K_RMS * rb, "c": 0.01}, auto)
    C.check("t", {"b": [10.0, 0.1, 0.12]}, auto)            # one wild realization: the median decides
    with pytest.raises(AssertionError):
        C.check("t", {"a": 0.051}, auto)
    with pytest.raises(AssertionError):
        C.check("t", {"b": [1.01 * C.K_RMS * rb] * 3}, auto)
    with pytest.raises(AssertionError, match="noise"):      # within every bound, but RHO > RHO_MAX
        C.check("t", {"a": [0.04, 0.045, 0.05], "b": [0.05, 0.2, 0.1]}, auto)
    C.check("t", {"h": 0.9}, auto, skip=["h"])
