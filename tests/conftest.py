"""Test configuration: puts the product package and the oracle on sys.path and
registers the ``gpu`` marker (tests that need an MI355X)."""
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "multimodal-deepfake-detection_amd")
for p in (PKG, REPO):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(REPO, "tests", "golden")

# The autocast reference of the bf16 contract (tests/bf16_contract.py) runs the oracle graph through
# MIOpen; its default find mode compiles and times every applicable solver for every new convolution
# shape on a fresh box (most of the bench-size bf16 test's ~3 minutes).  FAST: immediate mode, one
# kernel per shape.  (Test infrastructure only: the xcp path under test makes no MIOpen call.)
os.environ.setdefault("MIOPEN_FIND_MODE", "FAST")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP) device")


def has_gpu():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(scope="session")
def golden():
    import numpy as np

    cache = {}

    def load(name):
        if name not in cache:
            cache[name] = dict(np.load(os.path.join(GOLDEN, name), allow_pickle=False))
        return cache[name]
    return load


@pytest.fixture(scope="session")
def gpu():
    if not has_gpu():
        pytest.skip("no GPU")
    import torch
    return torch.device("cuda:0")
