"""Build-time invariants of the HIP sources that no GPU run can see (CPU: compiles to assembly)."""
import os
import shutil
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(not os.path.exists("/opt/rocm/bin/hipcc") and not shutil.which("hipcc"), reason="hipcc absent")
def test_nt4p_accumulators_stay_in_named_agprs():
    """The 4-wave persistent NT kernel names its 256 accumulator AGPRs in inline asm; that is only
    safe while the compiler never allocates an AGPR itself (no spill to AGPR, no scratch) --
    tools/check_nt4p_regs.py asserts it on the gfx950 assembly."""
    r = subprocess.run([sys.executable, os.path.join(REPO, "tools", "check_nt4p_regs.py")], capture_output=True,
                       text=True)
    assert r.returncode == 0, r.stdout + r.stderr


@pytest.mark.skipif(not os.path.exists("/opt/rocm/bin/hipcc") and not shutil.which("hipcc"), reason="hipcc absent")
def test_hot_kernels_do_not_spill():
    """No scratch (spilled registers) in the hot kernels: GEMMs, depthwise, fused unit backward,
    BN-backward apply (tools/check_spills.py)."""
    r = subprocess.run([sys.executable, os.path.join(REPO, "tools", "check_spills.py")], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
