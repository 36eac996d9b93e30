"""The bf16 gradient-norm contract of SURVEY.md §8(c) and its measured exceptions.

Contract: in bf16 mode every parameter's gradient norm is within 5e-2 (relative) of the
reference's fp32 CPU value (tests/golden, captured from the reference itself).

Exceptions: the parameters listed in OVER exceed it, each with the error measured on the
MI355X (the engine is deterministic: the same inputs give the same bits on every run and
box) and the bound asserted for it (1.25 x the measured error).  They are the BatchNorm
affine gradients of the stem and of the first blocks -- dgamma = sum(dz * zhat), dbeta =
sum(dz) over up to 256 x 147^2 pixels, nearly cancelling sums of bf16 gradients -- and, at the
16-clip batch, the last head layers, whose ReLU masks flip under the bf16 perturbation of the
features (the head is also checked against the oracle head on the GPU's own features at
1e-3).  PyTorch's own bf16 autocast of the same graph shows the same spread
(test_bf16_gradient_noise_vs_torch_autocast).

XCP_BF16_RECORD=1 prints every parameter above 5e-2 per tag without asserting (how the table
below was measured).
"""
import os

TOL = 5e-2
RECORD = os.environ.get("XCP_BF16_RECORD") == "1"

# tag -> {parameter: bound}; bound = 1.25 x the measured error (round 3, MI355X)
OVER = {
    'backbone64': {
        'bn1.weight': 0.161,
        'block2.rep.5.bias': 0.11,
        'block2.skipbn.bias': 0.11,
        'block1.rep.4.weight': 0.093,
        'block1.rep.1.weight': 0.089,
        'block2.rep.5.weight': 0.084,
        'bn2.weight': 0.077,
        'bn2.bias': 0.07,
        'block2.skipbn.weight': 0.068,
        'block1.skipbn.bias': 0.066,
        'block1.rep.4.bias': 0.065,
        'block1.rep.1.bias': 0.064,
    },
    'lstmv_b2t4_unfrozen': {
        'feature_extractor.bn2.bias': 0.132,
        'feature_extractor.block1.rep.4.weight': 0.114,
        'feature_extractor.bn2.weight': 0.095,
        'feature_extractor.bn1.weight': 0.092,
        'feature_extractor.block9.rep.2.weight': 0.082,
        'feature_extractor.block2.rep.2.bias': 0.082,
        'feature_extractor.block10.rep.2.weight': 0.081,
        'feature_extractor.block6.rep.2.bias': 0.071,
        'feature_extractor.block1.rep.1.weight': 0.069,
    },
    'lstmv_b4t16': {
        'feature_extractor.bn2.weight': 0.16,
        'feature_extractor.bn2.bias': 0.103,
        'feature_extractor.bn1.bias': 0.097,
        'feature_extractor.block7.rep.5.bias': 0.086,
        'feature_extractor.block1.rep.4.weight': 0.08,
        'feature_extractor.block5.rep.8.bias': 0.065,
        'feature_extractor.block6.rep.8.bias': 0.064,
        'feature_extractor.block2.rep.2.weight': 0.064,
    },
    'lstmv_b16t16': {
        'feature_extractor.bn1.weight': 0.285,
        'feature_extractor.bn2.weight': 0.11,
        'feature_extractor.block1.skipbn.weight': 0.093,
        'fc_layers.9.bias': 0.089,
        'feature_extractor.block3.rep.2.bias': 0.086,
        'fc_layers.9.weight': 0.079,
        'feature_extractor.block2.rep.5.weight': 0.074,
        'feature_extractor.bn1.bias': 0.069,
        'feature_extractor.block2.rep.2.weight': 0.067,
        'feature_extractor.block5.rep.2.weight': 0.067,
        'feature_extractor.block8.rep.8.weight': 0.067,
        'feature_extractor.block4.rep.2.bias': 0.065,
        'grad/lstm.bias_ih_l0': 0.527,
        'grad/fc_out.weight': 0.114,
    },
    'xception_c1_b4': {
        'bn2.weight': 0.349,
        'block1.rep.4.bias': 0.169,
        'block1.skipbn.bias': 0.169,
        'bn1.weight': 0.122,
        'bn2.bias': 0.117,
        'block1.rep.1.bias': 0.086,
        'block8.rep.5.bias': 0.078,
        'block1.skipbn.weight': 0.069,
        'grad/fc.weight': 0.137,
    },
    'xception_c2_b64': {
        'bn1.bias': 0.523,
        'bn1.weight': 0.165,
        'block1.rep.1.bias': 0.138,
        'block1.rep.1.weight': 0.097,
        'block2.skipbn.weight': 0.083,
        'bn2.weight': 0.075,
        'block4.rep.2.weight': 0.071,
        'conv1.weight': 0.063,
        'block3.rep.5.bias': 0.063,
        'block3.skipbn.bias': 0.063,
    },
}


def check(tag, errs, skip=()):
    """errs: {parameter: relative gradient-norm error vs the reference}; skip: names checked
    elsewhere.  Asserts the contract with this tag's exceptions."""
    over = sorted(((n, e) for n, e in errs.items() if e > TOL and n not in skip), key=lambda kv: -kv[1])
    print(f"\nbf16 gradient norms above {TOL} [{tag}]: {{" + ", ".join(f"{n!r}: {e:.4f}" for n, e in over) + "}")
    if RECORD:
        return
    table = OVER.get(tag, {})
    bad = [(n, round(e, 4), table.get(n, TOL)) for n, e in errs.items() if n not in skip and e > table.get(n, TOL)]
    assert not bad, f"bf16 gradient norms outside the contract [{tag}]: {bad}"
