"""A/B of patched variants of the persistent NT kernel (tile 3) at the middle-flow shape
(M = 256 x 19 x 19, 736 x 736, bf16, BN-statistics epilogue), each built from csrc/gemm.hip
into tools/exp/ (git-ignored), timed in interleaved rounds in one process.

  python tools/gemm_var.py build     # here
  python tools/gemm_var.py run [rounds]
"""
import ctypes
import os
import statistics
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
SRC = os.path.join(REPO, "multimodal-deepfake-detection_amd", "xcp", "csrc")
OUT = os.path.join(HERE, "exp")

ISSUE = "      __builtin_amdgcn_raw_ptr_buffer_load_lds(isA ? rA : rB, (__attribute__((address_space(3))) void*)(d + i * 1024),\n                                               16, o, 0, 0, 0);"


def variant(name):
    s = open(os.path.join(SRC, "gemm.hip")).read()
    s = s.replace('#include "common.h"\n', '#include "' + os.path.join(SRC, "common.h") + '"\n', 1)
    assert ISSUE in s
    aux = {"base": ("0", "0"), "a_nt": ("2", "0"), "ab_nt": ("2", "2"), "a_sc1": ("16", "0")}[name]
    new = ("      if (isA) __builtin_amdgcn_raw_ptr_buffer_load_lds(rA, (__attribute__((address_space(3))) void*)(d + i * 1024), "
           f"16, o, 0, 0, {aux[0]});\n"
           "      else __builtin_amdgcn_raw_ptr_buffer_load_lds(rB, (__attribute__((address_space(3))) void*)(d + i * 1024), "
           f"16, o, 0, 0, {aux[1]});")
    s = s.replace(ISSUE, new)
    return s


NAMES = ["base", "a_nt", "ab_nt", "a_sc1"]


def build():
    os.makedirs(OUT, exist_ok=True)
    for n in NAMES:
        src = os.path.join(OUT, f"gemm_var_{n}.hip")
        open(src, "w").write(variant(n))
        so = os.path.join(OUT, f"libgemm_var_{n}.so")
        r = subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "-shared", "--offload-arch=gfx950",
                            "-munsafe-fp-atomics", src, "-o", so], capture_output=True, text=True)
        if r.returncode:
            raise SystemExit(r.stderr)
        print("built", so)


def run():
    import torch
    sys.path[:0] = [os.path.join(REPO, "multimodal-deepfake-detection_amd"), REPO]
    from xcp import _lib
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    dev = torch.device("cuda:0")
    M, C = 256 * 361, 736
    g = torch.Generator(device=dev).manual_seed(0)
    A = torch.randn(M, C, device=dev, generator=g).bfloat16()
    B = (torch.randn(C, C, device=dev, generator=g) / 27).bfloat16()
    Y = torch.empty_like(A)
    st = torch.empty(((M + 127) // 128) * 2 * C, device=dev)
    s = torch.cuda.current_stream().cuda_stream
    z = (0, 0, 0, 0, 0, 1, 0)
    libs = {}
    for n in NAMES:
        lib = ctypes.CDLL(os.path.join(OUT, f"libgemm_var_{n}.so"))
        lib.xcp_gemm_nt.argtypes = _lib.SIGNATURES["xcp_gemm_nt"]
        lib.xcp_gemm_nt.restype = ctypes.c_int
        libs[n] = lib

    def timeit(fn, iters=20):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / iters * 1e3

    res = {(n, t): [] for n in NAMES for t in (0, 3)}
    for _ in range(rounds):
        for (n, t) in res:
            lib = libs[n]
            res[(n, t)].append(timeit(lambda: lib.xcp_gemm_nt(1, A.data_ptr(), C, B.data_ptr(), C, Y.data_ptr(), C, M,
                                                              C, C, st.data_ptr(), *z, t, s)))
    ref = None
    for (n, t), v in res.items():
        med = statistics.median(v)
        print(f"{n:8s} tile={t}  median {med:7.1f} us  min {min(v):7.1f}  frac {2.0 * M * 728 * 728 / med / 1e6 / 2500:.3f}",
              flush=True)


if __name__ == "__main__":
    {"build": build, "run": run}[sys.argv[1]]()
