"""GEMM ablation experiments, kept out of the product library: variants of csrc/gemm.hip
built from patched copies of the source into tools/exp/ (git-ignored .so files that still
travel to the GPU box) and timed at the middle-flow shape (M = 256 x 19 x 19, 728 x 728).

  python tools/gemm_exp.py build        # here (hipcc cross-compiles gfx950)
  python tools/gemm_exp.py run          # on the GPU box

Variants: base (unpatched), nomfma (MFMAs replaced by a register sink that keeps the
fragment reads alive), noload (LDS-DMA issues removed: LDS holds stale data), nomfma+noload,
nobar2 / noload_nobar2 (timing only: the barrier after each MFMA cluster removed), noepi /
noload_noepi (timing only: the epilogue replaced by a register sink).
GEMM_EXP_VARIANTS=a,b selects a subset.
"""
import ctypes
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
SRC = os.path.join(REPO, "multimodal-deepfake-detection_amd", "xcp", "csrc")
OUT = os.path.join(HERE, "exp")

FAKE_MFMA = r'''
XCP_DEV f32x4 xcp_fake_mfma(bf16x8 a, bf16x8 b, f32x4 c, int, int, int) {
  asm volatile("" :: "v"(a), "v"(b));
  return c;
}
'''
FAKE_GLDS = r'''
XCP_DEV void xcp_fake_glds(const void __attribute__((address_space(1)))* p, void __attribute__((address_space(3)))* d,
                           int, int, int) {
  asm volatile("" :: "v"(p));
}
XCP_DEV void xcp_fake_bload(__amdgpu_buffer_rsrc_t r, void __attribute__((address_space(3)))* d, int, unsigned o, int,
                            int, int) {
  asm volatile("" :: "v"(o));
}
'''
VARIANTS = {"base": (), "nomfma": ("mfma",), "noload": ("load",), "nomfma_noload": ("mfma", "load"),
            "nobar2": ("bar2",), "noload_nobar2": ("load", "bar2"), "noepi": ("epi",), "noload_noepi": ("load", "epi")}
SEL = os.environ.get("GEMM_EXP_VARIANTS")   # comma-separated subset to build / run


def patched(kinds):
    s = open(os.path.join(SRC, "gemm.hip")).read()
    head = '#include "common.h"\n'
    extra = ""
    if "mfma" in kinds:
        s = s.replace("__builtin_amdgcn_mfma_f32_16x16x32_bf16(", "xcp_fake_mfma(")
        extra += FAKE_MFMA
    if "bar2" in kinds:   # timing only: NT256 phases without the barrier after each MFMA cluster
        old = "    mfma_q(ih, b, jh);\n    __builtin_amdgcn_s_setprio(0);\n    __builtin_amdgcn_s_barrier();\n"
        assert old in s
        s = s.replace(old, "    mfma_q(ih, b, jh);\n    __builtin_amdgcn_s_setprio(0);\n")
    if "epi" in kinds:    # timing only: NT256 epilogue replaced by a sink that keeps every MFMA alive
        old = "  epilogue256_regs(acc, a, m0, n0, wr, wc, fr, fg);\n}"
        assert old in s
        s = s.replace(old, """  float sink = 0.f;
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) sink += acc[i][j][0] + acc[i][j][1] + acc[i][j][2] + acc[i][j][3];
  if (sink == 1234.5f) reinterpret_cast<float*>(a.stats)[threadIdx.x] = sink;
}""")
    if "load" in kinds:
        s = s.replace("__builtin_amdgcn_global_load_lds(", "xcp_fake_glds(")
        s = s.replace("__builtin_amdgcn_raw_ptr_buffer_load_lds(", "xcp_fake_bload(")
        extra += FAKE_GLDS
    s = s.replace(head, '#include "' + os.path.join(SRC, "common.h") + '"\n' + extra, 1)
    return s


def build():
    os.makedirs(OUT, exist_ok=True)
    for name, kinds in VARIANTS.items():
        if SEL and name not in SEL.split(","):
            continue
        src = os.path.join(OUT, f"gemm_{name}.hip")
        open(src, "w").write(patched(kinds))
        so = os.path.join(OUT, f"libgemm_{name}.so")
        cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "-shared", "--offload-arch=gfx950",
               "-munsafe-fp-atomics", src, "-o", so]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode:
            raise SystemExit(r.stderr)
        print("built", so)


def run():
    import torch
    sys.path[:0] = [os.path.join(REPO, "multimodal-deepfake-detection_amd"), REPO]
    from xcp import _lib
    dev = torch.device("cuda:0")
    M, C = 256 * 361, 728
    g = torch.Generator(device=dev).manual_seed(0)
    X = torch.randn(M, C, device=dev, generator=g).to(torch.bfloat16)
    D = torch.randn(M, C, device=dev, generator=g).to(torch.bfloat16)
    Wp = (torch.randn(C, C, device=dev, generator=g) / 27).to(torch.bfloat16)
    Y = torch.empty_like(X)
    st = torch.empty(((M + 127) // 128) * 2 * C, device=dev)
    stream = torch.cuda.current_stream().cuda_stream

    def timeit(fn, iters=20):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(iters):
            fn()
        e.record()
        torch.cuda.synchronize()
        return s.elapsed_time(e) / iters * 1e3

    for name in VARIANTS:
        if SEL and name not in SEL.split(","):
            continue
        lib = ctypes.CDLL(os.path.join(OUT, f"libgemm_{name}.so"))
        for fn in ("xcp_gemm_nt", "xcp_gemm_tn", "xcp_gemm_tn_rows_per_split"):
            getattr(lib, fn).argtypes = _lib.SIGNATURES[fn]
            getattr(lib, fn).restype = ctypes.c_int
        rps = lib.xcp_gemm_tn_rows_per_split(1, 0, M, C, C, 0)
        S = (M + rps - 1) // rps
        P = torch.empty(S * C * C, device=dev)
        z = (0, 0, 0, 0, 0, 1, 0)
        for tile in (2, 0):
            t = timeit(lambda: lib.xcp_gemm_nt(1, X.data_ptr(), C, Wp.data_ptr(), C, Y.data_ptr(), C, M, C, C,
                                               st.data_ptr(), *z, tile, stream))
            print(f"{name:14s} nt tile={tile}  {t:8.1f} us  {2.0 * M * C * C / t / 1e6:7.1f} TFLOP/s", flush=True)
        t = timeit(lambda: lib.xcp_gemm_tn(1, D.data_ptr(), C, X.data_ptr(), C, P.data_ptr(), M, C, C, S, rps, *z, 0,
                                           stream))
        print(f"{name:14s} tn S={S}     {t:8.1f} us  {2.0 * M * C * C / t / 1e6:7.1f} TFLOP/s", flush=True)
        if name == "base":   # 128-B aligned rows: the same 728-channel problem stored with a 768 stride
            L = 768
            Xp = torch.zeros(M, L, device=dev, dtype=torch.bfloat16)
            Xp[:, :C] = X
            Dp = torch.zeros(M, L, device=dev, dtype=torch.bfloat16)
            Dp[:, :C] = D
            Wpp = torch.zeros(C, L, device=dev, dtype=torch.bfloat16)
            Wpp[:, :C] = Wp
            Yp = torch.empty(M, L, device=dev, dtype=torch.bfloat16)
            for tile in (2,):
                t = timeit(lambda: lib.xcp_gemm_nt(1, Xp.data_ptr(), L, Wpp.data_ptr(), L, Yp.data_ptr(), L, M, C, C,
                                                   st.data_ptr(), *z, tile, stream))
                print(f"{name:14s} nt tile={tile} ld768  {t:8.1f} us  {2.0 * M * C * C / t / 1e6:7.1f} TFLOP/s",
                      flush=True)
            t = timeit(lambda: lib.xcp_gemm_tn(1, Dp.data_ptr(), L, Xp.data_ptr(), L, P.data_ptr(), M, C, C, S, rps,
                                               *z, 0, stream))
            print(f"{name:14s} tn S={S} ld768 {t:8.1f} us  {2.0 * M * C * C / t / 1e6:7.1f} TFLOP/s", flush=True)
            # full 768 problem (padded channels computed): what a padded layout would run
            t = timeit(lambda: lib.xcp_gemm_nt(1, Xp.data_ptr(), L, Wpp.data_ptr(), L, Yp.data_ptr(), L, M, L, L,
                                               st.data_ptr(), *z, 2, stream))
            print(f"{name:14s} nt 768x768      {t:8.1f} us", flush=True)
            del Xp, Dp, Wpp, Yp


if __name__ == "__main__":
    {"build": build, "run": run}[sys.argv[1]]()
