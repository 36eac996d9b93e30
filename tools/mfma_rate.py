"""MFMA issue-rate microbenchmark at one wave per SIMD (256-thread workgroups, one per CU):
cycles per group of 128 MFMA-cycles (8 x v_mfma_f32_16x16x32_bf16 or 4 x 32x32x16, accumulators
in fixed AGPRs; s_memtime around the loop, median over waves) bare, with 2 (or 4) ds_read_b128 per
group, bunched or spread between the MFMAs, consumed two groups later, and with 2 LDS-DMA issues
per group (the 4-wave NT kernel's k-step densities).
  python tools/mfma_rate.py build   # here
  python tools/mfma_rate.py run     # GPU box
"""
import ctypes
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, "exp")
SO = os.path.join(OUT, "libmfma_rate.so")
ITER = 64


def source():
    mf = []
    for t in range(64):
        n = 4 * t
        mf.append(f'    case {t}: asm volatile("v_mfma_f32_16x16x32_bf16 a[{n}:{n+3}], %0, %1, a[{n}:{n+3}]" :: "v"(b), "v"(a) : '
                  + ", ".join(f'"a{n+k}"' for k in range(4)) + "); break;")
    return r'''#include <hip/hip_runtime.h>
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
template <int V> struct IC { static constexpr int value = V; constexpr operator int() const { return V; } };
template <int B, int E, typename F> __device__ __forceinline__ void sfor(F&& f) {
  if constexpr (B < E) { f(IC<B>{}); sfor<B + 1, E>(f); } }
template <int t> __device__ __forceinline__ void mf(const bf16x8& b, const bf16x8& a) {
  switch (t) {
''' + "\n".join(mf) + r'''
  }
}
template <int t> __device__ __forceinline__ void mf32(const bf16x8& b, const bf16x8& a) {   // 32x32x16, acc a[16t:16t+15]
  if constexpr (t == 0) asm volatile("v_mfma_f32_32x32x16_bf16 a[0:15], %0, %1, a[0:15]" :: "v"(b), "v"(a) : "a0","a1","a2","a3","a4","a5","a6","a7","a8","a9","a10","a11","a12","a13","a14","a15");
  else if constexpr (t == 1) asm volatile("v_mfma_f32_32x32x16_bf16 a[16:31], %0, %1, a[16:31]" :: "v"(b), "v"(a) : "a16","a17","a18","a19","a20","a21","a22","a23","a24","a25","a26","a27","a28","a29","a30","a31");
  else if constexpr (t == 2) asm volatile("v_mfma_f32_32x32x16_bf16 a[32:47], %0, %1, a[32:47]" :: "v"(b), "v"(a) : "a32","a33","a34","a35","a36","a37","a38","a39","a40","a41","a42","a43","a44","a45","a46","a47");
  else asm volatile("v_mfma_f32_32x32x16_bf16 a[48:63], %0, %1, a[48:63]" :: "v"(b), "v"(a) : "a48","a49","a50","a51","a52","a53","a54","a55","a56","a57","a58","a59","a60","a61","a62","a63");
}
// V: 0 bare 16x16 (64 accs); 1 bunched 2 reads / 8 MFMA; 2 spread 1 read / 4 MFMA; 3 spread 3 reads / 8;
//    4 = 2 + 2 DMA / 8 spread; 5 32x32x16 bare; 6 32x32x16 spread 1 read / 2 MFMA; 7 = 6 + 2 DMA / 4 MFMA
template <int V>
__global__ __launch_bounds__(256) void rate(const bf16x8* in, long long* out, int iters) {
  __shared__ __attribute__((aligned(16))) char lds[65536];
  const int lane = threadIdx.x & 63;
  bf16x8 r[4];
  for (int k = 0; k < 4; ++k) r[k] = in[threadIdx.x + 256 * k];
  for (int i = threadIdx.x; i < 65536 / 16; i += 256) reinterpret_cast<uint4*>(lds)[i] = make_uint4(i, 0, 0, 0);
  __syncthreads();
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)in, (short)0, 0x7fffffff, 0x00020000);
  auto rd = [&](int k, int off) { return *reinterpret_cast<const bf16x8*>(lds + ((off * 1024 + lane * 16) & 49151)); };
  auto dma = [&](int i) {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)(lds + 49152 + (i & 7) * 1024), 16, lane * 16 + i * 1024, 0, 0, 0);
  };
  long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
    // 8 groups of 128 MFMA-cycles; a group's MFMAs use r[g % 4] (read two groups earlier)
    sfor<0, 8>([&](auto g) {
      constexpr int cur = g % 4, nxt = (g + 2) % 4;
      if constexpr (V == 0) {
        sfor<0, 8>([&](auto j) { mf<g * 8 + j>(r[cur], r[(cur + 1) % 4]); });
      } else if constexpr (V == 1) {
        r[nxt] = rd(nxt, g * 2);
        __builtin_amdgcn_sched_barrier(0);
        sfor<0, 8>([&](auto j) { mf<g * 8 + j>(r[cur], r[(cur + 1) % 4]); });
        __builtin_amdgcn_sched_barrier(0);
        r[(nxt + 1) % 4] = rd(nxt, g * 2 + 1);   // (a second read into the other half of the pair)
      } else if constexpr (V == 2 || V == 3 || V == 4) {
        sfor<0, 2>([&](auto h) {
          if constexpr (V == 4) dma(g * 2 + h);
          r[(nxt + h) % 4] = rd(nxt, g * 2 + h);
          if constexpr (V == 3) { bf16x8 z = rd(0, g * 2 + h + 9); asm volatile("" :: "v"(z)); }
          __builtin_amdgcn_sched_barrier(0);
          sfor<0, 4>([&](auto j) { mf<g * 8 + h * 4 + j>(r[cur], r[(cur + 1) % 4]); });
          __builtin_amdgcn_sched_barrier(0);
        });
      } else if constexpr (V == 5) {
        sfor<0, 4>([&](auto j) { mf32<j>(r[cur], r[(cur + 1) % 4]); });
      } else {
        sfor<0, 2>([&](auto h) {
          if constexpr (V == 7) dma(g * 2 + h);
          r[(nxt + h) % 4] = rd(nxt, g * 2 + h);
          __builtin_amdgcn_sched_barrier(0);
          sfor<0, 2>([&](auto j) { mf32<h * 2 + j>(r[cur], r[(cur + 1) % 4]); });
          __builtin_amdgcn_sched_barrier(0);
        });
      }
    });
  }
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  long long t1 = __builtin_amdgcn_s_memtime();
  float s = 0.f;
  for (int k = 0; k < 4; ++k) s += (float)r[k][0];
  if (lane == 0) out[blockIdx.x * 4 + (threadIdx.x >> 6)] = (t1 - t0) + (s == 12345.f ? 1 : 0);
}
extern "C" int run_rate(int v, const void* in, long long* out, int iters) {
  const bf16x8* p = (const bf16x8*)in;
  switch (v) {
    case 0: hipLaunchKernelGGL(rate<0>, dim3(256), dim3(256), 0, 0, p, out, iters); break;
    case 1: hipLaunchKernelGGL(rate<1>, dim3(256), dim3(256), 0, 0, p, out, iters); break;
    case 2: hipLaunchKernelGGL(rate<2>, dim3(256), dim3(256), 0, 0, p, out, iters); break;
    case 3: hipLaunchKernelGGL(rate<3>, dim3(256), dim3(256), 0, 0, p, out, iters); break;
    case 4: hipLaunchKernelGGL(rate<4>, dim3(256), dim3(256), 0, 0, p, out, iters); break;
    case 5: hipLaunchKernelGGL(rate<5>, dim3(256), dim3(256), 0, 0, p, out, iters); break;
    case 6: hipLaunchKernelGGL(rate<6>, dim3(256), dim3(256), 0, 0, p, out, iters); break;
    default: hipLaunchKernelGGL(rate<7>, dim3(256), dim3(256), 0, 0, p, out, iters); break;
  }
  return (int)hipDeviceSynchronize();
}
'''


def build():
    os.makedirs(OUT, exist_ok=True)
    src = os.path.join(OUT, "mfma_rate.hip")
    open(src, "w").write(source())
    r = subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "-shared", "--offload-arch=gfx950", src, "-o", SO],
                       capture_output=True, text=True)
    if r.returncode:
        raise SystemExit(r.stderr[-3000:])
    print("built", SO)


def run():
    import statistics as S
    import torch
    lib = ctypes.CDLL(SO)
    inp = torch.randn(8192, device="cuda").bfloat16()
    out = torch.zeros(1024, dtype=torch.int64, device="cuda")
    names = ["16x16 bare", "16x16 2rd bunched", "16x16 2rd spread", "16x16 4rd spread", "16x16 2rd+2dma",
             "32x32 bare", "32x32 2rd spread", "32x32 2rd+2dma"]
    for rep in range(2):
        for v, nm in enumerate(names):
            lib.run_rate(v, ctypes.c_void_p(inp.data_ptr()), ctypes.c_void_p(out.data_ptr()), ITER)
            c = out.cpu().tolist()
            n = 64 if v < 5 else 32   # MFMAs per iteration (32x32x16: 4 per 128-cycle group)
            print(f"{nm:20s} cycles per 128-cycle group: median {S.median(c) / (8 * ITER):7.1f}  min {min(c) / (8 * ITER):7.1f}"
                  f"   ({S.median(c) / (n * ITER):5.2f} per MFMA)", flush=True)


if __name__ == "__main__":
    {"build": build, "run": run}[sys.argv[1]]()
