"""Cycle accounting of the 4-wave NT kernel (tile 5 / 6) at the middle-flow shape: a patched copy of
csrc/gemm.hip (tools/exp/, git-ignored) in which every wave reads the shader clock (s_memtime) only
where its LDS reads are already drained (so the stamp's lgkmcnt wait changes nothing): after the
first k-step's lgkmcnt(0), after the middle vmcnt(0) + barrier, and at the end of the K-tile.
Sums per phase over the K-loop go to a buffer of its own; prints the per-K-tile mean cycles of
(first k-step, middle wait + barrier, second k-step), the prologue and the epilogue.

  python tools/gemm_stamps4.py build     # here
  python tools/gemm_stamps4.py run       # GPU box
"""
import ctypes
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
SRC = os.path.join(REPO, "multimodal-deepfake-detection_amd", "xcp", "csrc")
OUT = os.path.join(HERE, "exp")
VARIANTS = {   # experiment variants: (old, new) source replacements inside the kernel (timing only)
    "base": [],
    # fragment registers held one group longer (no ds_read into a register an in-flight MFMA reads)
    "hold": [("      __builtin_amdgcn_sched_barrier(0);\n    });\n    asm volatile(\"s_waitcnt lgkmcnt(0)\"",
              "      __builtin_amdgcn_sched_barrier(0);\n      if constexpr (g > 0) asm volatile(\"\" :: \"v\"(fa[g - 1]));\n"
              "    });\n    asm volatile(\"s_waitcnt lgkmcnt(0)\""),
             ("      static_for<4, 8>([&](auto j) { mfma_fixed<false, 32 + (g - 8) * 4 + (j - 4)>(fb1[j + 0], fa[g]); });\n"
              "      __builtin_amdgcn_sched_barrier(0);\n",
              "      static_for<4, 8>([&](auto j) { mfma_fixed<false, 32 + (g - 8) * 4 + (j - 4)>(fb1[j + 0], fa[g]); });\n"
              "      __builtin_amdgcn_sched_barrier(0);\n      asm volatile(\"\" :: \"v\"(fa[g - 1]));\n")],
    # no LDS-DMA issues (results meaningless)
    "nodma": [("      issue1(op, G + 2, k2, nx, i0);\n", ""), ("      issue1(op, G + 2, k2, nx, i0 + 1);\n", "")],
    # no fragment reads in the loop (results meaningless)
    "noreads": [("      fa[g + 2] = frag(sa, aoff, (g + 2) & 7, (g + 2) >> 3);\n      fb1[g] = frag(sb, boff, g, 1);\n",
                 "      fa[g + 2] = fa[g];\n      fb1[g] = fb0[g];\n"),
                ("      fa[g + 2] = g + 2 < 16 ? frag(sa, aoff, (g + 2) & 7, 1) : frag(sa1, aoff, g - 14, 0);\n", "      fa[g + 2] = fa[g];\n"),
                ("      fb0[g - 8] = frag(sb1, boff, g - 8, 0);\n", "      fb0[g - 8] = fb1[g - 8];\n")],
}


def so_path(variant):
    return os.path.join(OUT, f"libgemm_stamps4_{variant}.so")
NS = 8   # values per wave


def patched(variant="base"):
    s = open(os.path.join(SRC, "gemm.hip")).read()
    s = s.replace('#include "common.h"\n', '#include "' + os.path.join(SRC, "common.h") + '"\n'
                  "__device__ long long* g_stamps;\n", 1)
    k0 = s.index("template <bool STATS>\n__global__ __launch_bounds__(256) void gemm_nt4p_kernel")
    k1 = s.index("// Weight gradient: P[s]")
    k = s[k0:k1]
    reps = [
        ("  __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0), as a real s_waitcnt (see the loop's end)\n",
         "  __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0), as a real s_waitcnt (see the loop's end)\n"
         "  long long T0_ = __builtin_amdgcn_s_memtime(), tp_ = T0_, s1_ = 0, s2_ = 0, s3_ = 0, s4_ = 0;\n"),
        ("    asm volatile(\"s_waitcnt lgkmcnt(0)\" ::: \"memory\");   // B(G) and A(G-1) fully read by this wave\n",
         "    asm volatile(\"s_waitcnt lgkmcnt(0)\" ::: \"memory\");   // B(G) and A(G-1) fully read by this wave\n"
         "    { long long n_ = __builtin_amdgcn_s_memtime(); s1_ += n_ - tp_; tp_ = n_; }\n"),
        ("    __builtin_amdgcn_s_barrier();\n    // k-step 1:",
         "    __builtin_amdgcn_s_barrier();\n    { long long n_ = __builtin_amdgcn_s_memtime(); s2_ += n_ - tp_; tp_ = n_; }\n    // k-step 1:"),
        ("    __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0)\n    if (++kt == nk) {\n",
         "    __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0)\n"
         "    { long long n_ = __builtin_amdgcn_s_memtime(); s3_ += n_ - tp_; tp_ = n_; }\n    if (++kt == nk) {\n"),
        ("      set_offsets(t + nwg, vnA, vnB);\n    }\n  }\n",
         "      set_offsets(t + nwg, vnA, vnB);\n"
         "      __builtin_amdgcn_s_waitcnt(0xC07F);\n"
         "      { long long n_ = __builtin_amdgcn_s_memtime(); s4_ += n_ - tp_; tp_ = n_; }\n    }\n  }\n"
         "  const long long TX_ = __builtin_amdgcn_s_memtime();\n"
         "  if (lane == 0) { long long* o_ = g_stamps + ((long)blockIdx.x * 4 + w) * " + str(NS) + ";\n"
         "    o_[0] = T0_; o_[1] = total; o_[2] = s1_; o_[3] = s2_; o_[4] = s3_; o_[5] = s4_; o_[6] = TX_ - T0_; o_[7] = nk; }\n"),
    ]
    for a, b in reps + VARIANTS[variant]:
        assert a in k, a[:70]
        k = k.replace(a, b, 1)
    s = s[:k0] + k + s[k1:]
    s += ('\nextern "C" int xcp_set_stamps(long long* p) {\n'
          '  return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), &p, sizeof(p));\n}\n')
    return s


def build():
    os.makedirs(OUT, exist_ok=True)
    for v in VARIANTS:
        src = os.path.join(OUT, f"gemm_stamps4_{v}.hip")
        open(src, "w").write(patched(v))
        r = subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "-shared", "--offload-arch=gfx950",
                            "-munsafe-fp-atomics", src, "-o", so_path(v)], capture_output=True, text=True)
        if r.returncode:
            raise SystemExit(r.stderr)
        print("built", so_path(v))


def run():
    import statistics as S
    import torch
    sys.path[:0] = [os.path.join(REPO, "multimodal-deepfake-detection_amd"), REPO]
    from xcp import _lib
    dev = torch.device("cuda:0")
    C = 736
    s = torch.cuda.current_stream().cuda_stream
    z = (0, 0, 0, 0, 0, 1, 0)
    for variant in (sys.argv[2:] or list(VARIANTS)):
        lib = ctypes.CDLL(so_path(variant))
        lib.xcp_gemm_nt.argtypes = _lib.SIGNATURES["xcp_gemm_nt"]
        lib.xcp_gemm_nt.restype = ctypes.c_int
        lib.xcp_set_stamps.argtypes = [ctypes.c_void_p]
        for stats in (False, True):
            M = 256 * 361
            g = torch.Generator(device=dev).manual_seed(0)
            A = torch.randn(M, C, device=dev, generator=g).bfloat16()
            B = (torch.randn(C, C, device=dev, generator=g) / 27).bfloat16()
            Y = torch.empty_like(A)
            st = torch.empty(((M + 127) // 128) * 2 * C, device=dev)
            stamps = torch.zeros(256 * 4 * NS, device=dev, dtype=torch.int64)
            lib.xcp_set_stamps(ctypes.c_void_p(stamps.data_ptr()))
            sp = st.data_ptr() if stats else None
            for _ in range(20):
                lib.xcp_gemm_nt(1, A.data_ptr(), C, B.data_ptr(), C, Y.data_ptr(), C, M, C, C, sp, *z, 5, s)
            torch.cuda.synchronize()
            stamps.zero_()
            lib.xcp_gemm_nt(1, A.data_ptr(), C, B.data_ptr(), C, Y.data_ptr(), C, M, C, C, sp, *z, 5, s)
            torch.cuda.synchronize()
            v = stamps.view(-1, NS).cpu().double()
            v = v[v[:, 7] > 0]
            kts = v[:, 1]
            tiles_ = kts / v[:, 7]
            q = lambda x: f"median {S.median(x):8.0f}  min {min(x):8.0f}  max {max(x):8.0f}"   # noqa: E731
            print(f"{variant}: stats={stats} waves {len(v)}  (cycles; loop phases per K-tile, epilogue per tile)")
            print("  k-step 0 + reads    ", q(list(v[:, 2] / kts)))
            print("  middle wait+barrier ", q(list(v[:, 3] / kts)))
            print("  k-step 1 + issues   ", q(list(v[:, 4] / kts)))
            print("  epilogue per tile   ", q(list(v[:, 5] / tiles_)))
            print("  whole loop          ", q(list(v[:, 6])), flush=True)


if __name__ == "__main__":
    {"build": build, "run": run}[sys.argv[1]]()
