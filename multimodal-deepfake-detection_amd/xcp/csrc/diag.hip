// Diagnostic: the shader clock the chip holds under a bf16 MFMA load, measured in-kernel
// (MI355X_MICROARCH.md "DVFS give-back" item 6: clock = d(shader cycle counter) /
// d(100 MHz real-time counter)).  Not on the training path: bench.py runs it before the
// warm-up (idle chip) and right after the timed steps (the chip as the step left it), so a
// bench line shows when a box holds a lower clock than another.
//
// One 256-thread workgroup per CU (one wave per SIMD), each wave a back-to-back
// v_mfma_f32_16x16x32_bf16 chain on non-trivial operands (zero operands hold a higher clock,
// item 1).  Lane 0 of wave 0 writes (cycles, real-time ticks) of its loop to out[2 * block];
// the accumulators feed a never-taken store so the loop is kept.
#include "common.h"

namespace {

__global__ __launch_bounds__(256) void clock_probe_kernel(long long* out, int iters) {
  const int lane = threadIdx.x & 63;
  bf16x8 a, b;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    a[i] = (bf16)(0.25f + 0.01f * (float)((lane * 7 + i * 3 + blockIdx.x) & 31));
    b[i] = (bf16)(-0.5f + 0.02f * (float)((lane * 5 + i * 11) & 63));
  }
  f32x4 acc[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  __syncthreads();
  const long long c0 = clock64(), r0 = wall_clock64();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc[j], 0, 0, 0);
  }
  const float s = acc[0][0] + acc[1][1] + acc[2][2] + acc[3][3];
  const long long c1 = clock64(), r1 = wall_clock64();
  if (threadIdx.x == 0) {
    out[2 * blockIdx.x] = c1 - c0;
    out[2 * blockIdx.x + 1] = r1 - r0;
  }
  if (s == 1234.5f) out[2 * gridDim.x + threadIdx.x] = 1;   // never true for these operands
}

// Streaming copy, 16 B per lane, 4 loads in flight per thread (the guide's float4 copy, which
// measured 6.29 TB/s on MI355X): the "measured copy peak" the depthwise fractions are quoted
// against.  n16 = 16-B units, a multiple of 1024.
__global__ __launch_bounds__(256) void stream_copy_kernel(const uint4* __restrict__ in, uint4* __restrict__ out) {
  const long base = (long)blockIdx.x * 1024 + threadIdx.x;
  uint4 v[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) v[k] = in[base + k * 256];
#pragma unroll
  for (int k = 0; k < 4; ++k) out[base + k * 256] = v[k];
}

// One-GPU stand-in for a bucket all-reduce (xcp.ddp proxy mode, profiles/r06_ddp_proxy.txt): `gridDim.x`
// workgroups (RCCL's channel blocks) stream the bucket's bytes through the chip once (read + write) and
// then hold their CUs until `ticks` of the 100 MHz real-time clock have passed since each started -- the
// time the ring all-reduce would take on the links.  rec (uint64 [3], pre-set to {~0, 0, 0}): the first
// workgroup start, the last workgroup start and the last workgroup end, on the same clock as
// stamp_kernel (so a stand-in that waits for CUs the weight-gradient stream holds shows it).
__global__ __launch_bounds__(256) void comm_proxy_kernel(const uint4* __restrict__ in, uint4* __restrict__ out, long n16,
                                                         long long ticks, unsigned long long* rec) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) {
    atomicMin(rec, t0);
    atomicMax(rec + 1, t0);
  }
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n16; i += (long)gridDim.x * 256) out[i] = in[i];
  while ((long long)(__builtin_amdgcn_s_memrealtime() - t0) < ticks) __builtin_amdgcn_s_sleep(8);
  __syncthreads();
  if (threadIdx.x == 0) atomicMax(rec + 2, (unsigned long long)__builtin_amdgcn_s_memrealtime());
}

// one 100 MHz real-time stamp into *out (a marker on a stream, on comm_proxy_kernel's clock)
__global__ __launch_bounds__(64) void stamp_kernel(unsigned long long* out) {
  if (threadIdx.x == 0) atomicMax(out, (unsigned long long)__builtin_amdgcn_s_memrealtime());
}

}  // namespace

extern "C" {

int xcp_comm_proxy(const void* in, void* out, long n16, int blocks, long long ticks, unsigned long long* rec,
                   hipStream_t stream) {
  if (n16 < 0 || blocks <= 0 || blocks > 1024 || ticks < 0 || !rec) return XCP_EINVAL;
  hipLaunchKernelGGL(comm_proxy_kernel, dim3(blocks), dim3(256), 0, stream, reinterpret_cast<const uint4*>(in),
                     reinterpret_cast<uint4*>(out), n16, ticks, rec);
  return (int)hipGetLastError();
}

int xcp_stamp(unsigned long long* out, hipStream_t stream) {
  if (!out) return XCP_EINVAL;
  hipLaunchKernelGGL(stamp_kernel, dim3(1), dim3(64), 0, stream, out);
  return (int)hipGetLastError();
}

int xcp_stream_copy(const void* in, void* out, long n16, hipStream_t stream) {
  if (n16 <= 0 || n16 % 1024) return XCP_EINVAL;
  hipLaunchKernelGGL(stream_copy_kernel, dim3((unsigned)(n16 / 1024)), dim3(256), 0, stream,
                     reinterpret_cast<const uint4*>(in), reinterpret_cast<uint4*>(out));
  return (int)hipGetLastError();
}

// out: DEVICE int64 [2 * blocks + 256]; see include/xcp.h
int xcp_clock_probe(long long* out, int blocks, int iters, hipStream_t stream) {
  if (blocks <= 0 || iters <= 0) return XCP_EINVAL;
  hipLaunchKernelGGL(clock_probe_kernel, dim3(blocks), dim3(256), 0, stream, out, iters);
  return (int)hipGetLastError();
}

}  // extern "C"
