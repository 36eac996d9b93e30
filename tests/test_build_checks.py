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


def _vregs(operand):
    """VGPR numbers named by one asm operand: v7 / v[4:7]."""
    import re
    m = re.fullmatch(r"v(\d+)", operand) or re.fullmatch(r"v\[(\d+):(\d+)\]", operand)
    if not m:
        return set()
    lo = int(m.group(1))
    hi = int(m.group(2)) if m.lastindex == 2 else lo
    return set(range(lo, hi + 1))


@pytest.mark.skipif(not os.path.exists("/opt/rocm/bin/hipcc") and not shutil.which("hipcc"), reason="hipcc absent")
def test_sep_fwd_asm_loads_untouched_until_their_wait(tmp_path):
    """The fused block1 forward (csrc/sepfwd.hip) loads its look-ahead input rows with inline-asm
    global loads the compiler does not track; correctness needs every instruction between such a load
    and the next vmcnt wait to leave its destination registers alone (a copy or a spill of one would read
    the register before the data lands).  Checked on the gfx950 assembly of every instantiation, along
    every control-flow path from each load to the first vmcnt wait."""
    import re
    src = os.path.join(REPO, "multimodal-deepfake-detection_amd", "xcp", "csrc", "sepfwd.hip")
    out = tmp_path / "sepfwd.s"
    hipcc = "/opt/rocm/bin/hipcc" if os.path.exists("/opt/rocm/bin/hipcc") else shutil.which("hipcc")
    subprocess.run([hipcc, "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "--cuda-device-only", "-S", src, "-o",
                    str(out)], check=True, capture_output=True)
    lines = out.read_text().splitlines()
    labels = {l.split(":")[0]: k for k, l in enumerate(lines) if re.match(r"^\.LBB[^:\s]*:", l)}

    def instr(k):
        t = lines[k].strip()
        return "" if not t or t.startswith((";", ".")) or t.endswith(":") else t

    loads = 0
    for i, l in enumerate(lines):
        m = re.match(r"\s*global_load_dwordx4 (v\[\d+:\d+\]),", l)
        if not m:
            continue
        loads += 1
        regs = _vregs(m.group(1))
        # every path from the load (control flow followed through branches) until a vmcnt wait
        todo, seen = [i + 1], set()
        while todo:
            k = todo.pop()
            while k < len(lines) and k not in seen:
                seen.add(k)
                t = instr(k)
                if t.startswith("s_waitcnt") and "vmcnt" in t or t.startswith("s_endpgm"):
                    break
                if t.startswith("global_load_dwordx4"):
                    k += 1
                    continue
                if t:
                    ops = [o.strip() for o in t.split(None, 1)[1].split(",")] if " " in t else []
                    touched = set().union(*[_vregs(o) for o in ops]) if ops else set()
                    assert not (touched & regs), f"line {i}: {l.strip()} -> line {k}: {t}"
                if t.startswith("s_branch "):
                    k = labels[t.split()[1]]
                    continue
                if t.startswith("s_cbranch"):
                    todo.append(labels[t.split()[1]])
                k += 1
    assert loads >= 6 * 2, loads
