"""Build-time invariants of the HIP sources that no GPU run can see (CPU: compiles to assembly)."""
import os
import shutil
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(not os.path.exists("/opt/rocm/bin/hipcc") and not shutil.which("hipcc"), reason="hipcc absent")
def test_hot_kernels_do_not_spill():
    """No scratch (spilled registers) in the hot kernels: GEMMs, depthwise, fused unit backward,
    BN-backward apply (tools/check_spills.py)."""
    r = subprocess.run([sys.executable, os.path.join(REPO, "tools", "check_spills.py")], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
