// Depthwise 3x3 forward (stride 1, pad 1) for tiny frames, bf16.
//
// Reference op: SeparableConv2d.conv1 (Xception.py:41, called at :45) with the producer's
// BatchNorm + ReLU applied to its input (Block.rep, Xception.py:61-87), at the frame sizes
// of the 64^2 audio family (XceptionLSTMA.py:46): 8x8, 4x4 and 2x2 after the entry flow.
#include "common.h"

namespace {

typedef float f2 __attribute__((ext_vector_type(2)));

XCP_DEV f2 fma2(f2 a, f2 b, f2 c) { return __builtin_elementwise_fma(a, b, c); }
XCP_DEV f2 max0(f2 a) { return __builtin_elementwise_max(a, f2(0.f)); }

// ---------------------------------------------------------------------------------
// Depthwise forward for tiny frames (W <= 8: the 4x4 middle flow and 2x2 / 8x8 layers of the
// 64^2 audio family, 1920 frames per step).  The tile kernel gives such a frame a whole
// workgroup and a mostly-halo LDS tile (42 staged pixels for 16 outputs at 4x4); here one
// thread owns 4 channels of one frame, walks its rows with a 3-row register window of
// activated fp32 pairs and reads every input element once (8-B loads, consecutive threads
// on consecutive channels) and writes every output once.
template <int ACT, int W>
__global__ __launch_bounds__(256) void dw_fwd_small_kernel(const bf16* __restrict__ X, bf16* __restrict__ Y,
                                                           const float* __restrict__ Wt, const float* __restrict__ scale,
                                                           const float* __restrict__ shift, int N, int H, int C) {
  const int CV = C >> 2;
  const long gi = (long)blockIdx.x * 256 + threadIdx.x;
  if (gi >= (long)N * CV) return;
  const int n = (int)(gi / CV), c0 = (int)(gi - (long)n * CV) * 4;
  f2 wt[9][2], sc[2], sh[2];
#pragma unroll
  for (int t = 0; t < 9; ++t) {
    const float4 a = *reinterpret_cast<const float4*>(Wt + (long)t * C + c0);
    wt[t][0] = f2{a.x, a.y};
    wt[t][1] = f2{a.z, a.w};
  }
  if constexpr (ACT == ACT_BNRELU) {
    const float4 a = *reinterpret_cast<const float4*>(scale + c0), b = *reinterpret_cast<const float4*>(shift + c0);
    sc[0] = f2{a.x, a.y};
    sc[1] = f2{a.z, a.w};
    sh[0] = f2{b.x, b.y};
    sh[1] = f2{b.z, b.w};
  }
  const bf16* Xn = X + (long)n * H * W * C + c0;
  bf16* Yn = Y + (long)n * H * W * C + c0;
  // Row h's raw pixels are fetched one step ahead of their use (fetch_row issues all W loads
  // with no branch between them and nothing waits on them until the next step's act_row), so
  // the loads of row r + 2 are in flight while row r is computed.
  uint2 nx[W];
  auto fetch_row = [&](int h) {
#pragma unroll
    for (int x = 0; x < W; ++x) nx[x] = *reinterpret_cast<const uint2*>(Xn + ((long)h * W + x) * C);
  };
  // row h as W + 2 activated columns (zero padding at both ends and outside the frame)
  auto act_row = [&](int h, f2 (&o)[W + 2][2]) {
    const bool ok = h < H;   // h >= 0 here
    o[0][0] = o[0][1] = o[W + 1][0] = o[W + 1][1] = f2(0.f);
#pragma unroll
    for (int x = 0; x < W; ++x) {
      const uint2 u = nx[x];
      f2 v0 = f2{__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u)};
      f2 v1 = f2{__uint_as_float(u.y << 16), __uint_as_float(u.y & 0xffff0000u)};
      if constexpr (ACT == ACT_BNRELU) {
        v0 = max0(fma2(v0, sc[0], sh[0]));
        v1 = max0(fma2(v1, sc[1], sh[1]));
      } else if constexpr (ACT == ACT_RELU) {
        v0 = max0(v0);
        v1 = max0(v1);
      }
      o[x + 1][0] = ok ? v0 : f2(0.f);
      o[x + 1][1] = ok ? v1 : f2(0.f);
    }
  };
  auto step = [&](int r, const f2 (&ra)[W + 2][2], const f2 (&rb)[W + 2][2], f2 (&rc)[W + 2][2]) {
    act_row(r + 1, rc);
    if (r + 2 < H) fetch_row(r + 2);   // uniform: r and H are the same for every thread
#pragma unroll
    for (int x = 0; x < W; ++x) {
      f2 o[2];
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        f2 a = ra[x][e] * wt[0][e];
        f2 b = rb[x][e] * wt[3][e];
        f2 c = rc[x][e] * wt[6][e];
#pragma unroll
        for (int kx = 1; kx < 3; ++kx) {
          a = fma2(ra[x + kx][e], wt[kx][e], a);
          b = fma2(rb[x + kx][e], wt[3 + kx][e], b);
          c = fma2(rc[x + kx][e], wt[6 + kx][e], c);
        }
        o[e] = (a + b) + c;
      }
      bf16x4 q;
      q[0] = (bf16)o[0][0];
      q[1] = (bf16)o[0][1];
      q[2] = (bf16)o[1][0];
      q[3] = (bf16)o[1][1];
      *reinterpret_cast<uint2*>(Yn + ((long)r * W + x) * C) = __builtin_bit_cast(uint2, q);
    }
  };
  f2 w0[W + 2][2], w1[W + 2][2], w2[W + 2][2];
#pragma unroll
  for (int x = 0; x < W + 2; ++x) w0[x][0] = w0[x][1] = f2(0.f);   // row -1: padding
  fetch_row(0);
  act_row(0, w1);
  if (1 < H) fetch_row(1);
  for (int r = 0; r < H; r += 3) {
    step(r, w0, w1, w2);
    if (r + 1 < H) step(r + 1, w1, w2, w0);
    if (r + 2 < H) step(r + 2, w2, w0, w1);
  }
}

template <int W>
void launch_small_w(int act, const bf16* x, bf16* y, const float* Wt, const float* scale, const float* shift, int N,
                    int H, int C, hipStream_t st) {
  const long threads = (long)N * (C / 4);
  const dim3 grid((unsigned)((threads + 255) / 256));
  if (act == ACT_NONE)
    hipLaunchKernelGGL((dw_fwd_small_kernel<ACT_NONE, W>), grid, dim3(256), 0, st, x, y, Wt, scale, shift, N, H, C);
  else if (act == ACT_RELU)
    hipLaunchKernelGGL((dw_fwd_small_kernel<ACT_RELU, W>), grid, dim3(256), 0, st, x, y, Wt, scale, shift, N, H, C);
  else
    hipLaunchKernelGGL((dw_fwd_small_kernel<ACT_BNRELU, W>), grid, dim3(256), 0, st, x, y, Wt, scale, shift, N, H, C);
}

}  // namespace

// Tiny-frame depthwise forward (bf16, W in {1, 2, 4, 8}); XCP_EUNSUPPORTED otherwise.
int xcp_internal_dw_fwd_small(int act, const void* X, void* Y, const float* Wt, const float* scale, const float* shift,
                              int N, int H, int W, int C, hipStream_t st) {
  if (C % 8) return XCP_EUNSUPPORTED;
  const bf16* x = (const bf16*)X;
  bf16* y = (bf16*)Y;
  switch (W) {
    case 1: launch_small_w<1>(act, x, y, Wt, scale, shift, N, H, C, st); break;
    case 2: launch_small_w<2>(act, x, y, Wt, scale, shift, N, H, C, st); break;
    case 4: launch_small_w<4>(act, x, y, Wt, scale, shift, N, H, C, st); break;
    case 8: launch_small_w<8>(act, x, y, Wt, scale, shift, N, H, C, st); break;
    default: return XCP_EUNSUPPORTED;
  }
  return (int)hipGetLastError();
}
