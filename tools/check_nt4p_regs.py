"""Build-time check of the 4-wave persistent NT kernel (gemm_nt4p_kernel, csrc/gemm.hip): its
accumulators live in AGPRs a0-a255 named by inline asm, which is only safe while the compiler's
own code never touches an AGPR.  Compiles gemm.hip to gfx950 assembly and asserts, for both
instantiations: no VGPR spill and no scratch use, VGPRs well below 256, AGPR count 256, and no
AGPR access except the kernel's own MFMAs (a[4T:4T+3]) and epilogue reads (v_accvgpr_read_b32).

usage: python tools/check_nt4p_regs.py      (exit status 1 on a violation)
"""
import os
import re
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(os.path.dirname(HERE), "multimodal-deepfake-detection_amd", "xcp", "csrc", "gemm.hip")
VGPR_MAX = 232


def check():
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "gemm.s")
        r = subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950",
                            "--cuda-device-only", "-S", SRC, "-o", out, "-Rpass-analysis=kernel-resource-usage"],
                           capture_output=True, text=True)
        if r.returncode:
            raise SystemExit(r.stderr)
        asm = open(out).read()
    errs = []
    names = sorted(set(re.findall(r"^(\S*gemm_nt4p_kernel\S*):", asm, re.M)))
    if len(names) != 2:
        errs.append(f"expected 2 gemm_nt4p_kernel instantiations, found {names}")
    for name in names:
        i = asm.index(name + ":")
        j = asm.index(".Lfunc_end", i)
        body = [l.strip() for l in asm[i:j].split("\n") if l.strip() and not l.strip().startswith((";", "."))]
        for l in body:
            op = l.split()[0]
            if op.startswith("scratch_") or op.startswith("buffer_store_dword") and "off, s[0:3]" in l:
                errs.append(f"{name}: scratch access: {l}")
            if re.search(r"\ba\[?\d", l) and not (op == "v_mfma_f32_16x16x32_bf16" or op == "v_accvgpr_read_b32"):
                errs.append(f"{name}: compiler-generated AGPR use: {l}")
        vg = re.search(re.escape(name) + r"\.num_vgpr, (\d+)", asm)
        ag = re.search(re.escape(name) + r"\.num_agpr, (\d+)", asm)
        if not vg or int(vg.group(1)) > VGPR_MAX:
            errs.append(f"{name}: VGPRs {vg.group(1) if vg else '?'} > {VGPR_MAX}")
        if not ag or int(ag.group(1)) != 256:
            errs.append(f"{name}: AGPRs {ag.group(1) if ag else '?'} != 256")
        mf = sum(1 for l in body if l.startswith("v_mfma"))
        print(f"{name}: VGPRs {vg.group(1) if vg else '?'} AGPRs {ag.group(1) if ag else '?'} MFMAs {mf}")
    for e in errs[:20]:
        print("ERROR", e)
    return not errs


if __name__ == "__main__":
    sys.exit(0 if check() else 1)
