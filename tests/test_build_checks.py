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
    buffer loads the compiler does not track; correctness needs every instruction between such a load
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
        m = re.match(r"\s*(?:global|buffer)_load_dwordx4 (v\[\d+:\d+\]),", l)
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
                if t.startswith(("global_load_dwordx4", "buffer_load_dwordx4")):
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


def _compiler_vmcnt0_in_loops(lines, name_filter):
    """{kernel: [(line, instruction after the wait)]}: compiler-inserted (not inline asm) s_waitcnt with
    vmcnt(0) inside a loop (between a label and a backward branch to it) of each matching kernel."""
    import re
    out = {}
    k = 0
    while k < len(lines):
        m = re.match(r"^(_Z\S+):", lines[k])
        if not m:
            k += 1
            continue
        j = k
        while j < len(lines) and not lines[j].startswith(".Lfunc_end"):
            j += 1
        body = lines[k:j]
        if name_filter(m.group(1)):
            labels = {x.split(":")[0]: i for i, x in enumerate(body) if re.match(r"^\.LBB\S+:", x)}
            loops = []
            for i, x in enumerate(body):
                b = re.match(r"\s*s_(?:c)?branch\w*\s+(\.LBB\S+)", x)
                if b and b.group(1) in labels and labels[b.group(1)] < i:
                    loops.append((labels[b.group(1)], i))
            bad = [(i, body[i + 1].strip()) for i, x in enumerate(body)
                   if "s_waitcnt" in x and "vmcnt(0)" in x and "ASMSTART" not in body[i - 1]
                   and any(a <= i <= e for a, e in loops)]
            out[m.group(1)] = bad
        k = max(j, k + 1)
    return out


@pytest.mark.skipif(not os.path.exists("/opt/rocm/bin/hipcc") and not shutil.which("hipcc"), reason="hipcc absent")
def test_dma_pipelines_not_drained_by_compiler_waits(tmp_path):
    """The LDS-DMA pipelined kernels keep their look-ahead loads in flight: no compiler-inserted
    vmcnt(0) inside their loops (hipcc adds one ahead of an LDS access it cannot prove disjoint from an
    in-flight DMA -- a ds_read_tr builtin, an access after a second __shared__ object gave the accesses
    alias scopes, a compiler-visible global load in the prologue -- and it drains the look-ahead every
    iteration).  GEMMs (NT / TN 256x256), stem conv2 forward / dgrad / weight gradient, the depthwise
    backward's occupancy-4 forms (plain and asm ring reads, with and without the residual)."""
    import re
    hipcc = "/opt/rocm/bin/hipcc" if os.path.exists("/opt/rocm/bin/hipcc") else shutil.which("hipcc")
    csrc = os.path.join(REPO, "multimodal-deepfake-detection_amd", "xcp", "csrc")
    checks = {
        "gemm.hip": lambda n: re.search(r"gemm_(nt256p|nt256k64|tn256)_kernel", n),
        "conv3.hip": lambda n: "conv3x3" in n,
        # dw_bwd_lds_kernel<T, ACT, RES, ROLL=false, BD=1, MINW, SKIP=false, BNRES=false, ASMRD>
        "dwconv.hip": lambda n: re.search(r"dw_bwd_lds_kernelI(DF16b|f)Li\dELb[01]ELb0ELi1ELi[34]ELb0ELb0ELb[01]E", n),
    }
    procs = {}
    for f in checks:
        out = tmp_path / (f + ".s")
        procs[f] = (out, subprocess.Popen([hipcc, "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "--cuda-device-only",
                                           "-S", os.path.join(csrc, f), "-o", str(out)],
                                          stdout=subprocess.PIPE, stderr=subprocess.PIPE))
    for f, (out, p) in procs.items():
        _, err = p.communicate()
        assert p.returncode == 0, err.decode()[-2000:]
        found = _compiler_vmcnt0_in_loops(out.read_text().splitlines(), checks[f])
        assert found, f"{f}: no kernel matched"
        bad = {k: v for k, v in found.items() if v}
        assert not bad, f"{f}: {bad}"
