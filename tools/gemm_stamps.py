"""In-kernel timestamps of the persistent NT kernel (tile 3) at the middle-flow shape: a patched
copy of csrc/gemm.hip (tools/exp/, git-ignored) whose wave 0 / lane 0 writes the 100 MHz
real-time counter at kernel entry and, per tile, after the first K-tile's wait + barrier, after
the K-loop, and after the epilogue's stores are issued, into a buffer of its own (no output
value reads it).  Prints the per-phase distribution over workgroups and tiles.

  python tools/gemm_stamps.py build     # here
  python tools/gemm_stamps.py run       # GPU box
"""
import ctypes
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
SRC = os.path.join(REPO, "multimodal-deepfake-detection_amd", "xcp", "csrc")
OUT = os.path.join(HERE, "exp")
SO = os.path.join(OUT, "libgemm_stamps.so")
MAXT = 8   # tiles per workgroup recorded
NST = 1 + 3 * MAXT


def patched():
    s = open(os.path.join(SRC, "gemm.hip")).read()
    s = s.replace('#include "common.h"\n', '#include "' + os.path.join(SRC, "common.h") + '"\n'
                  "__device__ long long* g_stamps;\n"
                  f"#define XCP_STAMP(k) do {{ if (threadIdx.x == 0 && (k) < {NST}) "
                  f"g_stamps[(long)blockIdx.x * {NST} + (k)] = wall_clock64(); }} while (0)\n", 1)
    reps = [("  int t = slot;\n  if (t >= tiles) return;\n",
             "  int t = slot;\n  XCP_STAMP(0);\n  int it_ = 0;\n  if (t >= tiles) return;\n"),
            ("    __builtin_amdgcn_s_barrier();\n    if (wr == 1) __builtin_amdgcn_s_barrier();\n    // one 64-deep K-tile",
             "    __builtin_amdgcn_s_barrier();\n    if (wr == 1) __builtin_amdgcn_s_barrier();\n    XCP_STAMP(1 + 3 * it_);\n"
             "    // one 64-deep K-tile"),
            ("    if (wr == 0) __builtin_amdgcn_s_barrier();   // every wave is done reading both ring slots\n",
             "    if (wr == 0) __builtin_amdgcn_s_barrier();   // every wave is done reading both ring slots\n"
             "    XCP_STAMP(2 + 3 * it_);\n"),
            ("    epilogue256_buf<STATS>(acc, a, rC, rS, cm0, cn0, wr, wc, fr, fg);\n",
             "    epilogue256_buf<STATS>(acc, a, rC, rS, cm0, cn0, wr, wc, fr, fg);\n    XCP_STAMP(3 + 3 * it_);\n"
             "    ++it_;\n")]
    for a, b in reps:
        assert a in s, a[:60]
        s = s.replace(a, b, 1)
    s += ('\nextern "C" int xcp_set_stamps(long long* p) {\n'
          '  return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), &p, sizeof(p));\n}\n')
    return s


def build():
    os.makedirs(OUT, exist_ok=True)
    src = os.path.join(OUT, "gemm_stamps.hip")
    open(src, "w").write(patched())
    r = subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "-shared", "--offload-arch=gfx950",
                        "-munsafe-fp-atomics", src, "-o", SO], capture_output=True, text=True)
    if r.returncode:
        raise SystemExit(r.stderr)
    print("built", SO)


def run():
    import torch
    sys.path[:0] = [os.path.join(REPO, "multimodal-deepfake-detection_amd"), REPO]
    from xcp import _lib
    dev = torch.device("cuda:0")
    lib = ctypes.CDLL(SO)
    lib.xcp_gemm_nt.argtypes = _lib.SIGNATURES["xcp_gemm_nt"]
    lib.xcp_gemm_nt.restype = ctypes.c_int
    lib.xcp_set_stamps.argtypes = [ctypes.c_void_p]
    M, C = int(os.environ.get("STAMP_M", 256 * 361)), 736
    g = torch.Generator(device=dev).manual_seed(0)
    A = torch.randn(M, C, device=dev, generator=g).bfloat16()
    B = (torch.randn(C, C, device=dev, generator=g) / 27).bfloat16()
    Y = torch.empty_like(A)
    st = torch.empty(((M + 127) // 128) * 2 * C, device=dev)
    stamps = torch.zeros(256 * NST, device=dev, dtype=torch.int64)
    lib.xcp_set_stamps(ctypes.c_void_p(stamps.data_ptr()))
    s = torch.cuda.current_stream().cuda_stream
    z = (0, 0, 0, 0, 0, 1, 0)
    for _ in range(20):   # warm clocks, then the recorded launch
        lib.xcp_gemm_nt(1, A.data_ptr(), C, B.data_ptr(), C, Y.data_ptr(), C, M, C, C, st.data_ptr(), *z, 3, s)
    torch.cuda.synchronize()
    stamps.zero_()
    lib.xcp_gemm_nt(1, A.data_ptr(), C, B.data_ptr(), C, Y.data_ptr(), C, M, C, C, st.data_ptr(), *z, 3, s)
    torch.cuda.synchronize()
    v = stamps.view(256, NST).cpu().double() * 0.01   # 100 MHz ticks -> us
    t0 = v[:, 0].min()
    import statistics as S
    fills, loops, epis, gaps = [], [], [], []
    loops0, loopsn, fill0 = [], [], []
    ends = []
    for w in range(256):
        prev = v[w, 0]
        for it in range(MAXT):
            a1, a2, a3 = v[w, 1 + 3 * it], v[w, 2 + 3 * it], v[w, 3 + 3 * it]
            if a1 == 0:
                break
            fills.append(a1 - prev)
            loops.append(a2 - a1)
            (loops0 if it == 0 else loopsn).append(a2 - a1)
            if it == 0:
                fill0.append(a1 - prev)
            epis.append(a3 - a2)
            prev = a3
        ends.append(prev - t0)
    q = lambda x: f"median {S.median(x):6.2f}  min {min(x):6.2f}  max {max(x):6.2f}"   # noqa: E731
    print("entry skew (us)      ", q(list(v[:, 0] - t0)))
    print("tile start wait (us) ", q(fills), " (first tile: entry -> K-tile 0 landed; later: prev epilogue -> landed)")
    print("K-loop (us)          ", q(loops))
    print("  first tile         ", q(loops0))
    print("  later tiles        ", q(loopsn))
    print("first fill (us)      ", q(fill0))
    print("epilogue issue (us)  ", q(epis))
    print("last stamp (us)      ", q(ends))


if __name__ == "__main__":
    {"build": build, "run": run}[sys.argv[1]]()
