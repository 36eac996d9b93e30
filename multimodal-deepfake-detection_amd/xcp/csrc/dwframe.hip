// Depthwise 3x3 forward (stride 1, pad 1) for small frames -- the 728-channel 19x19
// middle flow, the 10x10 exit flow and the 64^2 audio family -- as a persistent,
// double-buffered kernel whose inner loop is FMAs only.
//
// Reference op: SeparableConv2d.conv1 (Xception.py:41, called at :45) with the producer's
// BatchNorm + ReLU applied to its input (Block.rep, Xception.py:61-87).
//
// Why a separate kernel: depthwise 3x3 is VALU-bound on CDNA4 long before HBM (one VALU
// instruction per 4 cycles per SIMD; 9 FMAs per element at best), and the tile kernel
// (dwconv.hip) spends ~36 lane-ops per element re-unpacking and re-activating every bf16
// input in each of the 9 windows that read it.  Here one 512-thread workgroup per CU walks
// units (frame n, 32-channel group g).  LDS-DMA brings the bf16 halo tile of unit k+1 (with
// the group's taps and BatchNorm scale / shift) into one of two raw buffers while unit k is
// computed; at the start of a unit its raw tile is unpacked and activated ONCE into an fp32
// tile ((H+2) x (W+2) x 128 B; padding reads a NaN line, and max(NaN * s + t, 0) = 0).  Thread
// (row part p, column x, 4-channel vector v) walks the rows of its part with a 3 x 3 window
// of fp32 pairs (16-B LDS reads, packed v_pk_fma_f32 math in three independent chains) and
// writes 8 B per output pixel.  Every thread issues the same number of stores per unit
// (out-of-range lanes write a per-workgroup sink), so the DMA of the next unit is retired by
// a counted vmcnt that leaves the previous unit's stores in flight.  (Staging through
// registers instead made the compiler wait for every store before reusing them.)
//
// MEASURED SLOWER than the tile kernel and therefore off by default (xcp_tune knob 13):
// 111 us against 65 us (warm) / 124 against 82 us (cold caches) at 256 x 19 x 19 x 728.
// One workgroup per CU keeps only ~31 KB of loads in flight per CU (two units through LDS),
// against ~115 KB for the tile kernel's five resident workgroups, and the ~3 us load latency
// under full-chip load then bounds it (register staging, DMA staging and an L2 prefetch
// three units ahead all measured 105-135 us).  Kept, with its tests, as the measured
// alternative.
#include "common.h"

namespace {

constexpr int FG_CH = 32;                                  // channels per unit
constexpr int FG_MAXPX = 484;                              // (H+2)(W+2) up to a 20 x 20 frame
constexpr int FG_RAWPAR = 9 * 8 + 2 * 8;                   // 16-B pieces of taps + scale + shift
constexpr int FG_RAW = ((FG_MAXPX * 4 + FG_RAWPAR + 63) / 64) * 1024;   // bf16 tile + params, whole DMAs
constexpr int FG_TILE = FG_MAXPX * FG_CH * 4;              // fp32 tile
constexpr int FG_NTH = 512;

__device__ __attribute__((aligned(64))) uint4 g_fzero[4];
__device__ __attribute__((aligned(64))) uint4 g_fnan[4] = {{0x7fc07fc0u, 0x7fc07fc0u, 0x7fc07fc0u, 0x7fc07fc0u},
                                                          {0x7fc07fc0u, 0x7fc07fc0u, 0x7fc07fc0u, 0x7fc07fc0u},
                                                          {0x7fc07fc0u, 0x7fc07fc0u, 0x7fc07fc0u, 0x7fc07fc0u},
                                                          {0x7fc07fc0u, 0x7fc07fc0u, 0x7fc07fc0u, 0x7fc07fc0u}};   // bf16 qNaN
__device__ __attribute__((aligned(64))) uint2 g_fsink[256][FG_NTH];   // per-workgroup store sinks

typedef float f2 __attribute__((ext_vector_type(2)));

XCP_DEV f2 fma2(f2 a, f2 b, f2 c) { return __builtin_elementwise_fma(a, b, c); }
XCP_DEV f2 max0(f2 a) { return __builtin_elementwise_max(a, f2(0.f)); }

// s_waitcnt vmcnt(N) as a real S_WAITCNT (gfx9 encoding: vmcnt[3:0] | expcnt[6:4] |
// lgkmcnt[11:8] | vmcnt_hi[15:14]), visible to the compiler's own wait insertion
template <int N>
XCP_DEV void vmwait_n() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 15) | (0x7 << 4) | (0xF << 8) | ((N >> 4) << 14));
}

// retire everything but the `n` youngest VMEM operations (n <= 15)
XCP_DEV void wait_but_stores(int n) {
  switch (n) {
    case 1: vmwait_n<1>(); break;
    case 2: vmwait_n<2>(); break;
    case 3: vmwait_n<3>(); break;
    case 4: vmwait_n<4>(); break;
    case 5: vmwait_n<5>(); break;
    case 6: vmwait_n<6>(); break;
    case 7: vmwait_n<7>(); break;
    case 8: vmwait_n<8>(); break;
    case 9: vmwait_n<9>(); break;
    case 10: vmwait_n<10>(); break;
    case 11: vmwait_n<11>(); break;
    case 12: vmwait_n<12>(); break;
    case 13: vmwait_n<13>(); break;
    case 14: vmwait_n<14>(); break;
    case 15: vmwait_n<15>(); break;
    default: vmwait_n<0>(); break;
  }
}

// VAR (measurement only): 1 = no FMAs, 3 = no stores; PF: L2 prefetch three units ahead
template <int ACT, int VAR = 0, bool PF = true>
__global__ __launch_bounds__(FG_NTH) void dw_fwd_frame_kernel(const bf16* __restrict__ X, bf16* __restrict__ Y,
                                                              const float* __restrict__ Wt,
                                                              const float* __restrict__ scale,
                                                              const float* __restrict__ shift, int N, int H, int W,
                                                              int C, int G, int parts, int rp) {
  __shared__ __attribute__((aligned(16))) char raw[2][FG_RAW];
  __shared__ __attribute__((aligned(16))) char tile[FG_TILE];
  __shared__ __attribute__((aligned(16))) char pfsink[FG_NTH / 64][256];   // prefetch DMA lands here (unread)
  const int HP = H + 2, WP = W + 2;
  const int TC = HP * WP * 4;                      // 16-B bf16 chunks (8 channels) of a halo tile
  const int ninstr = (TC + FG_RAWPAR + 63) / 64;
  const int pofs = TC * 16;                        // params in a raw buffer: taps [9][32], scale, shift (fp32)
  const int units = N * G;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wsc = __builtin_amdgcn_readfirstlane(tid >> 6);
  const void* pad = ACT == ACT_NONE ? (const void*)g_fzero : (const void*)g_fnan;

  auto dma_unit = [&](int u, int b) {
    const int n = u / G, g = u - n * G;
    const bf16* Xn = X + (long)n * H * W * C;
    const int cg0 = g * FG_CH;
    for (int j = wsc; j < ninstr; j += FG_NTH / 64) {
      const int q = j * 64 + lane;
      const void* src = g_fzero;
      if (q < TC) {
        const int pp = q >> 2, c = cg0 + (q & 3) * 8;
        const int hy = pp / WP, hx = pp - hy * WP;
        const int h = hy - 1, w = hx - 1;
        src = (h >= 0 && h < H && w >= 0 && w < W && c < C) ? (const void*)(Xn + ((long)h * W + w) * C + c) : pad;
      } else if (q < TC + FG_RAWPAR) {
        const int r = q - TC, t = r >> 3, c = cg0 + (r & 7) * 4;   // t 0-8 taps, 9 scale, 10 shift
        const float* base = t < 9 ? Wt + (long)t * C : (t == 9 ? scale : shift);
        if (c < C) src = base + c;
      }
      __builtin_amdgcn_global_load_lds((const void __attribute__((address_space(1)))*)src,
                                       (void __attribute__((address_space(3)))*)(raw[b] + j * 1024), 16, 0, 0);
    }
  };
  // L2 prefetch of unit u's input pixels: one 4-B LDS-DMA per 64-B channel chunk (its line)
  // into a scratch row.  Issued after a unit's stores, so the counted waits never cover it.
  constexpr int PFI = 8;   // prefetch instructions per wave per unit (64 lanes each)
  auto prefetch = [&](int u) {
    const int n = u / G, g = u - n * G;
    const char* Xb = reinterpret_cast<const char*>(X + (long)n * H * W * C + g * FG_CH);
    const int HW = H * W;
#pragma unroll
    for (int i = 0; i < PFI; ++i) {
      const int q = (i * (FG_NTH / 64) + wsc) * 64 + lane;   // pixel
      const void* src = q < HW ? (const void*)(Xb + (long)q * C * 2) : (const void*)g_fzero;
      __builtin_amdgcn_global_load_lds((const void __attribute__((address_space(1)))*)src,
                                       (void __attribute__((address_space(3)))*)pfsink[wsc], 4, 0, 0);
    }
  };
  // raw bf16 tile -> activated fp32 tile (each element once)
  auto convert = [&](int b) {
    const char* rb = raw[b];
    const int cq = tid & 3;   // FG_NTH % 4 == 0: a thread's chunks share their 8 channels
    f2 sc[4], sh[4];
    if constexpr (ACT == ACT_BNRELU) {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const float4 a = *reinterpret_cast<const float4*>(rb + pofs + 9 * 128 + (cq * 8 + 4 * h) * 4);
        const float4 d = *reinterpret_cast<const float4*>(rb + pofs + 10 * 128 + (cq * 8 + 4 * h) * 4);
        sc[2 * h] = f2{a.x, a.y};
        sc[2 * h + 1] = f2{a.z, a.w};
        sh[2 * h] = f2{d.x, d.y};
        sh[2 * h + 1] = f2{d.z, d.w};
      }
    }
    for (int q = tid; q < TC; q += FG_NTH) {
      const uint4 u4 = *reinterpret_cast<const uint4*>(rb + q * 16);
      const unsigned wd[4] = {u4.x, u4.y, u4.z, u4.w};
      f2 v[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        v[e] = f2{__uint_as_float(wd[e] << 16), __uint_as_float(wd[e] & 0xffff0000u)};
        if constexpr (ACT == ACT_BNRELU) v[e] = max0(fma2(v[e], sc[e], sh[e]));
        else if constexpr (ACT == ACT_RELU) v[e] = max0(v[e]);
      }
      float4* d = reinterpret_cast<float4*>(tile + (q >> 2) * (FG_CH * 4) + (q & 3) * 32);
      d[0] = make_float4(v[0][0], v[0][1], v[1][0], v[1][1]);
      d[1] = make_float4(v[2][0], v[2][1], v[3][0], v[3][1]);
    }
  };

  const int G0 = gridDim.x;
  int u = blockIdx.x;
  if (u >= units) return;   // uniform
  dma_unit(u, 0);

  // this thread's item: part p, column x, 4-channel vector v
  const int ipp = W * 8;
  const int p = tid / ipp, x = (tid - p * ipp) >> 3, v = tid & 7;
  const bool live = p < parts;
  const int r0 = p * rp;

  for (int k = 0; u < units; ++k, u += G0) {
    if (k == 0 || VAR == 3) vmwait_n<0>();
    else wait_but_stores(rp + (PF && u + 2 * G0 < units ? PFI : 0));   // unit k's DMA landed; unit k-1's stores
                                                                         // and prefetch may fly
    lds_barrier();              // ... in every wave; every wave done with the fp32 tile
    if (u + G0 < units) dma_unit(u + G0, (k + 1) & 1);
    convert(k & 1);
    lds_barrier();
    const char* rb = raw[k & 1];
    const int n = u / G, g = u - n * G;
    const int c0 = g * FG_CH + v * 4;
    const bool cok = live && c0 < C;
    f2 wt[9][2];
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const float4 a = *reinterpret_cast<const float4*>(rb + pofs + t * 128 + v * 16);
      wt[t][0] = f2{a.x, a.y};
      wt[t][1] = f2{a.z, a.w};
    }
    auto load_row = [&](int hy, f2 (&o)[3][2]) {
#pragma unroll
      for (int dx = 0; dx < 3; ++dx) {
        const float4 a = *reinterpret_cast<const float4*>(tile + (hy * WP + x + dx) * (FG_CH * 4) + v * 16);
        o[dx][0] = f2{a.x, a.y};
        o[dx][1] = f2{a.z, a.w};
      }
    };
    f2 w0[3][2], w1[3][2], w2[3][2];
    const int hb = min(r0, H);   // halo row of input row r0 - 1
    load_row(hb, w0);
    load_row(hb + 1, w1);
    bf16* Yn = Y + (long)n * H * W * C;
    // output row r0 + i from window rows (ra, rb, rc) = halo rows r, r+1, r+2; rc is read here.
    // Exactly one store per step (out-of-range rows / lanes write the sink).
    auto step = [&](int i, const f2 (&ra)[3][2], const f2 (&rb2)[3][2], f2 (&rc)[3][2]) {
      const int r = r0 + i;
      load_row(min(r + 2, H + 1), rc);
      f2 o[2];
      if constexpr (VAR == 1) {
#pragma unroll
        for (int e = 0; e < 2; ++e) o[e] = ra[1][e] + rb2[1][e] + rc[1][e];
      } else {
        f2 oa[2], ob[2];
#pragma unroll
        for (int e = 0; e < 2; ++e) {
          oa[e] = ra[0][e] * wt[0][e];
          ob[e] = rb2[0][e] * wt[3][e];
        }
#pragma unroll
        for (int kx = 1; kx < 3; ++kx)
#pragma unroll
          for (int e = 0; e < 2; ++e) {
            oa[e] = fma2(ra[kx][e], wt[kx][e], oa[e]);
            ob[e] = fma2(rb2[kx][e], wt[3 + kx][e], ob[e]);
          }
#pragma unroll
        for (int e = 0; e < 2; ++e) {
          f2 oc = rc[0][e] * wt[6][e];
          oc = fma2(rc[1][e], wt[7][e], oc);
          oc = fma2(rc[2][e], wt[8][e], oc);
          o[e] = (oa[e] + ob[e]) + oc;
        }
      }
      bf16x4 q4;
      q4[0] = (bf16)o[0][0];
      q4[1] = (bf16)o[0][1];
      q4[2] = (bf16)o[1][0];
      q4[3] = (bf16)o[1][1];
      const bool ok = cok && r < H;
      uint2* dst = ok ? reinterpret_cast<uint2*>(Yn + ((long)r * W + x) * C + c0) : &g_fsink[blockIdx.x & 255][tid];
      if (VAR != 3) *dst = __builtin_bit_cast(uint2, q4);
      else asm volatile("" ::"v"(o[0][0]));
    };
    for (int i = 0; i < rp; i += 3) {
      step(i, w0, w1, w2);
      if (i + 1 < rp) step(i + 1, w1, w2, w0);
      if (i + 2 < rp) step(i + 2, w2, w0, w1);
    }
    if (PF && u + 3 * G0 < units) prefetch(u + 3 * G0);
  }
}


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
  // row h as W + 2 activated columns (zero padding at both ends and outside the frame)
  auto load_row = [&](int h, f2 (&o)[W + 2][2]) {
    o[0][0] = o[0][1] = o[W + 1][0] = o[W + 1][1] = f2(0.f);
#pragma unroll
    for (int x = 0; x < W; ++x) {
      if (h < 0 || h >= H) {
        o[x + 1][0] = o[x + 1][1] = f2(0.f);
        continue;
      }
      const uint2 u = *reinterpret_cast<const uint2*>(Xn + ((long)h * W + x) * C);
      f2 v0 = f2{__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u)};
      f2 v1 = f2{__uint_as_float(u.y << 16), __uint_as_float(u.y & 0xffff0000u)};
      if constexpr (ACT == ACT_BNRELU) {
        v0 = max0(fma2(v0, sc[0], sh[0]));
        v1 = max0(fma2(v1, sc[1], sh[1]));
      } else if constexpr (ACT == ACT_RELU) {
        v0 = max0(v0);
        v1 = max0(v1);
      }
      o[x + 1][0] = v0;
      o[x + 1][1] = v1;
    }
  };
  auto step = [&](int r, const f2 (&ra)[W + 2][2], const f2 (&rb)[W + 2][2], f2 (&rc)[W + 2][2]) {
    load_row(r + 1, rc);
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
  load_row(-1, w0);
  load_row(0, w1);
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

int g_dw_small = 1;   // xcp_tune knob 16: tiny-frame depthwise forward (1) or the tile kernel (0)

int g_dwf_var = 0;   // xcp_tune knob 14: measurement variants 1, 3 (see the kernel)

int launch_frame(int act, const bf16* x, bf16* y, const float* Wt, const float* scale, const float* shift, int N, int H,
                 int W, int C, hipStream_t st) {
  if ((H + 2) * (W + 2) > FG_MAXPX || W * 8 > FG_NTH || C % 8) return XCP_EUNSUPPORTED;
  int parts = FG_NTH / (W * 8);
  if (parts > H) parts = H;
  const int rp = (H + parts - 1) / parts;
  if (rp > 7) return XCP_EUNSUPPORTED;
  parts = (H + rp - 1) / rp;
  const int G = (C + FG_CH - 1) / FG_CH;
  static const int cus = [] {
    int d = 0, n = 0;
    if (hipGetDevice(&d) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, d) != hipSuccess)
      n = 0;
    return n > 0 ? n : 256;
  }();
  const int units = N * G;
  const dim3 grid(units < cus ? units : cus), block(FG_NTH);
#define XCP_FRAME(A, V) \
  hipLaunchKernelGGL((dw_fwd_frame_kernel<A, V>), grid, block, 0, st, x, y, Wt, scale, shift, N, H, W, C, G, parts, rp)
  if ((g_dwf_var >= 1 && g_dwf_var <= 3) && act == ACT_BNRELU) {
    if (g_dwf_var == 1) XCP_FRAME(ACT_BNRELU, 1);
    else if (g_dwf_var == 2)
      hipLaunchKernelGGL((dw_fwd_frame_kernel<ACT_BNRELU, 0, false>), grid, block, 0, st, x, y, Wt, scale, shift, N, H, W,
                         C, G, parts, rp);
    else XCP_FRAME(ACT_BNRELU, 3);
  } else if (act == ACT_NONE) {
    XCP_FRAME(ACT_NONE, 0);
  } else if (act == ACT_RELU) {
    XCP_FRAME(ACT_RELU, 0);
  } else {
    XCP_FRAME(ACT_BNRELU, 0);
  }
#undef XCP_FRAME
  return (int)hipGetLastError();
}

}  // namespace

int xcp_internal_dw_small(int v) {
  const int old = g_dw_small;
  if (v == 0 || v == 1) g_dw_small = v;
  return old;
}

// Tiny-frame depthwise forward (bf16, W in {1, 2, 4, 8}); XCP_EUNSUPPORTED otherwise.
int xcp_internal_dw_fwd_small(int act, const void* X, void* Y, const float* Wt, const float* scale, const float* shift,
                              int N, int H, int W, int C, hipStream_t st) {
  if (!g_dw_small || C % 8) return XCP_EUNSUPPORTED;
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

int xcp_internal_dwf_var(int v) {
  const int old = g_dwf_var;
  if (v >= 0 && v <= 3) g_dwf_var = v;
  return old;
}

// Small-frame depthwise forward (bf16); XCP_EUNSUPPORTED when the frame is too large.
int xcp_internal_dw_fwd_frame(int act, const void* X, void* Y, const float* Wt, const float* scale, const float* shift,
                              int N, int H, int W, int C, hipStream_t st) {
  return launch_frame(act, (const bf16*)X, (bf16*)Y, Wt, scale, shift, N, H, W, C, st);
}
