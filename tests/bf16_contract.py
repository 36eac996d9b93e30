"""The bf16 gradient contract of SURVEY.md §8(c), bounded by PyTorch's own bf16 noise.

Contract: in bf16 mode every parameter's gradient norm is within 5e-2 (relative, TOL) of the
reference's fp32 CPU value (tests/golden, captured from the reference itself) -- or, where bf16
arithmetic itself cannot get that close, within K_RMS x the RMS error of R_AUTO realizations of
PyTorch's own bf16 autocast of the same graph on the same inputs, computed in the same test process:

    bound(p) = max(TOL, K_RMS * rms_r err_autocast_r(p))

and the engine's error is the median of X_REAL realizations of its own (XSCALES, the first the
test's main run):

    median_j err_xcp_j(p) <= bound(p)

Both sides are draws of rounding noise with a per-parameter scale (largest for the BatchNorm affine
gradients of the stem and the first blocks -- dgamma = sum(dz * zhat), dbeta = sum(dz) over up to
256 x 147^2 pixels, nearly cancelling sums -- and for head layers whose ReLU masks flip under the
feature noise), so the bound is a statement about noise scales, and it has to hold for every one of
~150 parameters x 8 bf16 tests at once.  Round 3 bounded one engine draw by 1.25 x one measurement;
round 4 first by 2.5 x the worst of 6 autocast draws, which puts the false-failure rate of an
equally noisy engine at 0.6 % per parameter, i.e. a red suite on most kernel changes (it failed on a
summation-order change of the stem, block4.rep.8.weight 0.0551 against 0.0534).  Simulated
(half-normal draws, 4 M trials; RHO = engine / autocast noise scale): the RMS of 24 draws estimates
the autocast scale to +-15 %, the median of 3 engine draws has a tail P(> t) ~ 3 P(|Z| > t)^2, and at
K_RMS = 6 (K_STEM = 4 for the five stem parameters: 1e-8 at RHO = 1, 1.7e-4 at 1.5) a parameter fails by chance with probability < 1e-6 at RHO = 1, 7.5e-6 at 1.5, 3.5e-4 at 2
(R = 24), and 2.5e-6 / 1.4e-4 / 1.5e-3 with the bench size's R_AUTO_LARGE = 12; the measured RHO is
0.69-1.44 over the round-4 runs (profiles/r04_bf16_rho.txt, r04_stem_conv1_split.txt), i.e. family-wise well under 1 %, while an error many times the
noise -- a defect -- still fails.

How much noisier the engine is, is measured, not assumed: RHO = sqrt(mean_p median_j(err_xcp)^2 /
rms_r(err_autocast)^2 / MED3_M2) pools every parameter above a floor (a tight estimate: ~150
ratios), and is asserted <= RHO_MAX.  (Measured 0.69-1.44: the engine is about as noisy as autocast although it keeps
the residual stream -- block outputs and their gradients -- in bf16, where autocast's stays in fp32.)

The realizations are decorrelated without changing the answer: the input clip is scaled by c and
conv1's weight by 1/c (scaled_input; for the engine, its conv1.weight reloaded / c).  conv1 is
linear and has no bias, so in exact arithmetic its output, every later activation, the loss and
every gradient (including conv1's, through the 1/c) are independent of c -- fp64 agrees to 1e-15,
fp32 to its own rounding noise (<= 1.1e-3 on BN affine sums; test_bf16_contract_cpu.py) -- while
every bf16 rounding from the input on falls differently.  (Scaling the input alone relies on bn1's
scale invariance, which its eps breaks by up to 2 % on nearly cancelling BN gradients: not used.)

The autocast graph is the oracle's functional restatement of the reference
(oracle/xception_oracle.py) run on the GPU under torch.autocast("cuda", bfloat16) -- MIOpen /
hipBLASLt convolutions in bf16, BatchNorm in fp32 -- with the head / loss in fp32 as in the xcp
path.  It is test infrastructure (the checker); the path under test never calls it.

XCP_BF16_RECORD=1 prints every parameter above TOL with its bound and does not assert.
"""
import os

import numpy as np
import torch

TOL = 5e-2
K_RMS = 6.0
R_AUTO = 24
R_AUTO_LARGE = 12   # the bench-size (256-frame) config: an autocast realization there takes ~7 s
X_REAL = 3
RHO_MAX = 2.0     # measured 0.69-1.44 (round 4); an engine twice as noisy as autocast fails
# the stem's parameters (conv1 on the matrix cores with split-bf16 products, BN1 / BN2 fused into
# the conv kernels both ways, round 4) get a tighter per-parameter ceiling than K_RMS, so that a
# defect confined to one of them cannot hide in the pooled RHO (advisor round 4)
K_STEM = 4.0
STEM = {("conv1", "weight"), ("bn1", "weight"), ("bn1", "bias"), ("bn2", "weight"), ("bn2", "bias")}
RHO_FLOOR = 1e-3   # parameters whose autocast RMS error is below this carry no scale information
# input scales of the autocast realizations: 2^(frac(i * golden ratio) - 1/2), in [0.71, 1.41), no
# two equal or a power of two apart
SCALES = tuple(2.0 ** (((i * 0.6180339887498949) % 1.0) - 0.5) for i in range(1, R_AUTO + 1))
# the engine's realizations (the first is the test's main run)
XSCALES = (1.0, 1.1487, 0.8706)
RECORD = os.environ.get("XCP_BF16_RECORD") == "1"


def relerr(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


def autocast_errors(sd, loss_fn, ref_norms, ref_elem=None, trainable=None, R=R_AUTO):
    """PyTorch bf16 autocast realizations of the oracle graph.

    sd: {state_dict key: tensor on the GPU} (the initial state of the model under test);
    loss_fn(params, scale) -> scalar loss, the graph with its backbone under autocast and the
    input scaled by `scale`; ref_norms: {param: reference fp32 gradient norm};
    ref_elem: {param: reference fp32 gradient array} for element-wise checks; trainable:
    names that get gradients (default: the keys of ref_norms).
    Returns ({param: [norm rel err per realization]}, {param: [element-wise rel err ...]})."""
    trainable = set(ref_norms if trainable is None else trainable)
    norms = {n: [] for n in ref_norms}
    elem = {n: [] for n in (ref_elem or {})}
    import time
    for i, c in enumerate(SCALES[:R]):
        t0 = time.time()
        params = {k: (v.detach().clone().requires_grad_(True) if k in trainable else v.detach().clone())
                  for k, v in sd.items()}
        loss_fn(params, c).backward()
        if i < 2 or i == R - 1:
            torch.cuda.synchronize()
            print(f"autocast realization {i}: {time.time() - t0:.2f} s", flush=True)
        for n in norms:
            gn = params[n].grad.double().norm().item()
            norms[n].append(abs(gn - float(ref_norms[n])) / max(float(ref_norms[n]), 1e-30))
        for n in elem:
            elem[n].append(relerr(params[n].grad.cpu(), ref_elem[n]))
        del params
    torch.cuda.synchronize()
    return norms, elem


def scaled_input(params, x, c, prefix=""):
    """(params with conv1.weight -> conv1.weight / c, x * c): the same function of the leaves,
    different bf16 roundings."""
    q = dict(params)
    q[prefix + "conv1.weight"] = params[prefix + "conv1.weight"] / c
    return q, x * c


def rms(v):
    v = np.asarray(v, np.float64)
    return float(np.sqrt(np.mean(v * v))) if v.size else 0.0


def med(e):
    """the engine's error of a parameter: a number, or the median of its realizations"""
    return float(np.median(e)) if isinstance(e, (list, tuple)) else float(e)


def is_stem(name):
    """the Xception stem's conv1 / bn1 / bn2 (Xception.py:118-123) under any model prefix -- not a
    SeparableConv2d's depthwise `.conv1` (whose parent is a rep index or conv3 / conv4)"""
    parts = name.split(".")
    return tuple(parts[-2:]) in STEM and (len(parts) == 2 or not (parts[-3].isdigit() or parts[-3] in ("conv3", "conv4")))


def bound(name, auto):
    """max(TOL, K x the RMS autocast error of `name`), K = K_STEM for the stem's parameters and K_RMS
    otherwise (TOL when auto has no entry)."""
    if not auto or name not in auto or not auto[name]:
        return TOL
    return max(TOL, (K_STEM if is_stem(name) else K_RMS) * rms(auto[name]))


# E[median(|Z1|, |Z2|, |Z3|)^2] for standard normal Z (2e7-draw simulation): the median of three
# half-normal draws of scale s has mean square MED3_M2 * s^2
MED3_M2 = 0.7044


def rho(errs, auto):
    """pooled engine / autocast noise-scale ratio over the parameters with three engine realizations
    (their median, robust to one wild draw) and an autocast RMS above RHO_FLOOR: sqrt(mean_p
    med_x(p)^2 / rms_a(p)^2 / MED3_M2); (None, 0) when there are none"""
    r = [med(e) ** 2 / rms(auto[n]) ** 2 / MED3_M2 for n, e in errs.items()
         if isinstance(e, (list, tuple)) and len(e) == 3 and auto and n in auto and rms(auto[n]) > RHO_FLOOR]
    return (float(np.sqrt(np.mean(r))), len(r)) if r else (None, 0)


def check(tag, errs, auto=None, skip=()):
    """errs: {parameter: relative gradient-norm (or element-wise) error vs the reference, or the list
    of the engine's realizations}; auto: autocast_errors' per-parameter realizations (None: TOL for
    every parameter); skip: names checked elsewhere."""
    rows = sorted(((n, med(e), bound(n, auto)) for n, e in errs.items() if n not in skip), key=lambda r: -r[1])
    over = [r for r in rows if r[1] > TOL]
    print(f"\nbf16 errors above {TOL} [{tag}] (name, xcp median, bound, autocast rms): {{"
          + ", ".join(f"{n!r}: ({e:.4f}, {b:.4f}, {rms(auto[n]) if auto and n in auto else float('nan'):.4f})"
                      for n, e, b in over) + "}")
    ratio = None
    if auto:
        top = sorted(((n, e / max(rms(auto[n]), 1e-12)) for n, e, _ in rows if n in auto and e > TOL),
                     key=lambda r: -r[1])[:5]
        print(f"largest xcp / autocast-rms ratios among those [{tag}]:", [(n, round(x, 2)) for n, x in top])
        stem = [(n, round(med(e) / max(rms(auto[n]), 1e-12), 2)) for n, e in errs.items()
                if n not in skip and is_stem(n) and n in auto]
        print(f"stem xcp / autocast-rms ratios [{tag}]:", stem)
        ratio, npar = rho({n: e for n, e in errs.items() if n not in skip}, auto)
        if ratio is not None:
            print(f"engine / autocast noise-scale ratio RHO [{tag}]: {ratio:.3f} over {npar} parameters")
    if RECORD:
        return
    bad = [(n, round(e, 4), round(b, 4)) for n, e, b in rows if e > b]
    assert not bad, f"bf16 errors outside the contract [{tag}]: {bad}"
    assert ratio is None or ratio <= RHO_MAX, f"engine bf16 noise {ratio:.2f} x autocast's [{tag}] (max {RHO_MAX})"
