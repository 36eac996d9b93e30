// Fused forward of one entry-flow SeparableConv2d: depthwise 3x3 (stride 1, pad 1) followed by the
// 1x1 pointwise conv to 128 channels, with the BatchNorm batch statistics of the pointwise output --
// Xception.py:37-47 (SeparableConv2d.forward = pointwise(conv1(x))) for block1's two units
// (147^2: 64 -> 128, 128 -> 128), whose pointwise GEMMs (K = 64 / 128) are HBM-bound.
//
// Unfused, the depthwise output D is written by dw_fwd and read back by the GEMM; here it goes from
// the depthwise FMAs through LDS straight into the MFMAs (D is still written once: the unit's
// backward reads it).  Bytes per output pixel: CIN*2 (input) + CIN*2 (D) + 256 (Y), against
// 2*CIN*2 + CIN*2 + 256 for the two kernels.
//
// Persistent: one 512-thread workgroup per CU walks output rows (tiles = one row of one frame,
// consecutive rows of a round on one XCD, so the three staged input rows are shared in L2).  A tile
// is CIN / 32 jobs of one 32-channel slice each:
//   * the slice's 3 input rows (W + 2 pixels x 64 B, zero padding by out-of-range buffer offsets)
//     arrive by LDS-DMA into a 3-slot ring, two jobs ahead (no registers held for the prefetch);
//   * the input BatchNorm + ReLU of the previous unit is applied in place (padding kept zero) and
//     rounded to bf16, as dw_fwd's staging does;
//   * each lane computes 5 pixels x 2 channels of the depthwise conv from a 3 x 7 window, the same
//     fma chain per channel as dw_fwd_w2_kernel (so D is bitwise dw_fwd's), into an LDS tile
//     [160 pixels][32 channels];
//   * wave w accumulates Y[px][16w .. 16w+15] += D[px][slice] W[16w..][slice]^T over the 10 pixel
//     blocks with v_mfma_f32_16x16x32_bf16 (operands and K order as gemm_nt_kernel: Y bitwise);
//   * the D slice is stored with 16-B buffer stores; after the last slice Y is stored and its
//     bf16 values enter per-lane BN sums, which the workgroup writes as one partial row at the end.
// The ring is read and written by inline asm (a compiler-visible LDS access that may alias an
// LDS-DMA destination makes hipcc wait for every outstanding vector-memory operation), and every
// VMEM instruction is issued by every wave whatever its lanes' validity, so the counted waits are
// exact: at job j the wave waits for the LDS-DMA of job j with the stores of jobs j-2, j-1 and the
// LDS-DMA of jobs j+1, j+2 still allowed in flight.
#include "common.h"

namespace {

constexpr int SP_WMAX = 152;                              // widest frame
constexpr int SP_ROWPX = SP_WMAX + 2;                     // staged pixels per input row (with padding)
constexpr int SP_NIN_MAX = (12 * SP_ROWPX + 63) / 64;     // LDS-DMA instructions per slice (29)
constexpr int SP_SLOT = SP_NIN_MAX * 1024;                // ring slot bytes
constexpr int SP_PXB = 160;                               // pixel rows of the D tile (10 MFMA blocks)
constexpr int SP_XP = 80;                                 // D tile pitch (64 B + 16: conflict-free b128 reads)
constexpr int SP_WP = 272;                                // weight pitch (256 B + 16)
constexpr int SP_CO = 128;
constexpr int SP_SEG = 5;                                 // depthwise outputs per lane
constexpr unsigned SP_OOB = 0x80000000u;
constexpr int SP_REC = 0x7fffffff;
constexpr int SP_DW3 = 0x00020000;

typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef int i32x2 __attribute__((ext_vector_type(2)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

struct SepArgs {
  const bf16* X;        // [N][H][W][CIN] unit input (before the input transform)
  const float* scale;   // [CIN] input BN (ACT_BNRELU)
  const float* shift;
  const float* dwt;     // [9][CIN] depthwise taps
  const bf16* pw;       // [128][CIN] pointwise weight
  bf16* D;              // [N][H][W][CIN] depthwise output
  bf16* Y;              // [N][H][W][128] pointwise output
  float* part;          // [gridDim.x][2][128] BN partial sums of Y (nullptr: none)
  int N, H, W;
};

XCP_DEV void sp_vm_wait(int n) {   // s_waitcnt vmcnt(n), n in [0, 63]
  switch (n < 0 ? 0 : n > 63 ? 63 : n) {
#define SP_VMW(k) case k: asm volatile("s_waitcnt vmcnt(" #k ")" ::: "memory"); break;
    SP_VMW(0) SP_VMW(1) SP_VMW(2) SP_VMW(3) SP_VMW(4) SP_VMW(5) SP_VMW(6) SP_VMW(7)
    SP_VMW(8) SP_VMW(9) SP_VMW(10) SP_VMW(11) SP_VMW(12) SP_VMW(13) SP_VMW(14) SP_VMW(15)
    SP_VMW(16) SP_VMW(17) SP_VMW(18) SP_VMW(19) SP_VMW(20) SP_VMW(21) SP_VMW(22) SP_VMW(23)
    SP_VMW(24) SP_VMW(25) SP_VMW(26) SP_VMW(27) SP_VMW(28) SP_VMW(29) SP_VMW(30) SP_VMW(31)
    SP_VMW(32) SP_VMW(33) SP_VMW(34) SP_VMW(35) SP_VMW(36) SP_VMW(37) SP_VMW(38) SP_VMW(39)
    SP_VMW(40) SP_VMW(41) SP_VMW(42) SP_VMW(43) SP_VMW(44) SP_VMW(45) SP_VMW(46) SP_VMW(47)
    SP_VMW(48) SP_VMW(49) SP_VMW(50) SP_VMW(51) SP_VMW(52) SP_VMW(53) SP_VMW(54) SP_VMW(55)
    SP_VMW(56) SP_VMW(57) SP_VMW(58) SP_VMW(59) SP_VMW(60) SP_VMW(61) SP_VMW(62) SP_VMW(63)
#undef SP_VMW
  }
}

// ring accesses (inline asm: see the header)
XCP_DEV unsigned sp_rd32(const char* p) {
  unsigned v;
  asm volatile("ds_read_b32 %0, %1" : "=v"(v) : "v"((unsigned)(size_t)(const __attribute__((address_space(3))) char*)(p))
               : "memory");
  return v;
}
XCP_DEV u32x4 sp_rd128(const char* p) {
  u32x4 v;
  asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"((unsigned)(size_t)(const __attribute__((address_space(3))) char*)(p))
               : "memory");
  return v;
}
XCP_DEV void sp_wr128(char* p, u32x4 v) {
  asm volatile("ds_write_b128 %0, %1" :: "v"((unsigned)(size_t)(__attribute__((address_space(3))) char*)(p)), "v"(v)
               : "memory");
}
XCP_DEV void sp_lgkm0() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }
XCP_DEV void sp_barrier() {   // LDS-only workgroup barrier (no vmcnt wait)
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

XCP_DEV float sp_lo(unsigned u) { return __uint_as_float(u << 16); }
XCP_DEV float sp_hi(unsigned u) { return __uint_as_float(u & 0xffff0000u); }
XCP_DEV unsigned sp_pack(float a, float b) {
  bf16x4 q;
  q[0] = (bf16)a;
  q[1] = (bf16)b;
  const u16x4 r = __builtin_bit_cast(u16x4, q);
  return (unsigned)r[0] | ((unsigned)r[1] << 16);
}

template <int ACT, int CIN>
__global__ __launch_bounds__(512) void sep_fwd_kernel(SepArgs a) {
  constexpr int S = CIN / 32;   // slices (jobs) per tile
  __shared__ __attribute__((aligned(16))) char ring[3 * SP_SLOT];
  __shared__ __attribute__((aligned(16))) char sx[2][SP_PXB * SP_XP];
  __shared__ __attribute__((aligned(16))) char sw[SP_CO * SP_WP];
  __shared__ float sprm[2][CIN];
  __shared__ float stap[9][CIN];

  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 15, fg = lane >> 4;
  const int H = a.H, W = a.W;
  const int T = a.N * H;                      // tiles (frame rows)
  const int G = gridDim.x;
  const int slot_id = xcd_remap(blockIdx.x, G);
  const int ntiles = (T - slot_id + G - 1) / G;
  const int njobs = ntiles * S;
  const int rowb = (W + 2) * 64;              // staged row bytes
  const int nch = 12 * (W + 2);               // 16-B chunks per staged slice
  const int nin = (nch + 63) >> 6;            // LDS-DMA instructions per slice
  const int cnt = w < nin ? (nin - w + 7) >> 3 : 0;   // this wave's share

  const __amdgpu_buffer_rsrc_t rX = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16*>(a.X), (short)0, SP_REC, SP_DW3);
  const __amdgpu_buffer_rsrc_t rD = __builtin_amdgcn_make_buffer_rsrc(a.D, (short)0, SP_REC, SP_DW3);
  const __amdgpu_buffer_rsrc_t rY = __builtin_amdgcn_make_buffer_rsrc(a.Y, (short)0, SP_REC, SP_DW3);

  // ---- resident operands: the pointwise weight, the input BN affine, the taps
  for (int c = tid; c < SP_CO * (CIN / 8); c += 512) {
    const int r = c / (CIN / 8), k = c % (CIN / 8);
    *reinterpret_cast<uint4*>(sw + r * SP_WP + k * 16) = *reinterpret_cast<const uint4*>(a.pw + (long)r * CIN + k * 8);
  }
  for (int c = tid; c < CIN; c += 512) {
    sprm[0][c] = ACT == ACT_BNRELU ? a.scale[c] : 1.f;
    sprm[1][c] = ACT == ACT_BNRELU ? a.shift[c] : 0.f;
  }
  for (int c = tid; c < 9 * CIN; c += 512) stap[c / CIN][c % CIN] = a.dwt[c];
  __syncthreads();

  auto tile_of = [&](int j, int& n, int& h, int& s) {
    const int r = j / S;
    s = j - r * S;
    const int t = r * G + slot_id;
    n = t / H;
    h = t - n * H;
  };
  // LDS-DMA of job j's slice into ring slot j % 3 (every wave issues its cnt instructions; a job
  // past the end stages zeros)
  auto issue = [&](int j) {
    char* slot = ring + (j % 3) * SP_SLOT;
    int n = 0, h = 0, s = 0;
    const bool live = j < njobs;
    if (live) tile_of(j, n, h, s);
    for (int m = 0; m < cnt; ++m) {
      const int k = w + 8 * m;
      const int i = k * 64 + lane;
      const int row = i / (4 * (W + 2));
      const int rem = i - row * 4 * (W + 2);
      const int px = rem >> 2, q = rem & 3;
      const int hh = h - 1 + row, ww = px - 1;
      const bool ok = live && i < nch && hh >= 0 && hh < H && ww >= 0 && ww < W;
      const unsigned off = ok ? (unsigned)(((((long)n * H + hh) * W + ww) * CIN + s * 32 + q * 8) * 2) : SP_OOB;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rX, (__attribute__((address_space(3))) void*)(slot + k * 1024), 16, off, 0,
                                               0, 0);
    }
  };

  // depthwise lane map: channels 2*cl, 2*cl+1 of the slice; pixels x0 .. x0+4
  const int cl = tid & 15, x0 = (tid >> 4) * SP_SEG;
  int wcol[SP_SEG + 2];
#pragma unroll
  for (int k = 0; k < SP_SEG + 2; ++k) wcol[k] = min(x0 + k, W + 1) * 64 + cl * 4;

  f32x4 acc[10];
#pragma unroll
  for (int b = 0; b < 10; ++b) acc[b] = f32x4{0.f, 0.f, 0.f, 0.f};
  float s1[4] = {0.f, 0.f, 0.f, 0.f}, s2[4] = {0.f, 0.f, 0.f, 0.f};

  issue(0);
  issue(1);
  int st_prev1 = 0, st_prev2 = 0;   // store instructions of jobs j-1, j-2
  for (int j = 0; j < njobs; ++j) {
    issue(j + 2);
    sp_vm_wait(2 * cnt + st_prev1 + st_prev2);
    sp_barrier();   // job j's slice is in LDS for every wave
    int n, h, s;
    tile_of(j, n, h, s);
    char* slot = ring + (j % 3) * SP_SLOT;

    if constexpr (ACT != ACT_NONE) {   // input transform in place, padding stays zero
      const int q = tid & 3;
      float sc[8], sh[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        sc[e] = sprm[0][s * 32 + q * 8 + e];
        sh[e] = sprm[1][s * 32 + q * 8 + e];
      }
      u32x4 v[4];
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        const int c = tid + 512 * m;
        v[m] = sp_rd128(slot + min(c, nch - 1) * 16);
      }
      sp_lgkm0();
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        const int c = tid + 512 * m;
        const int row = c / (4 * (W + 2));
        const int px = (c - row * 4 * (W + 2)) >> 2;
        const int hh = h - 1 + row, ww = px - 1;
        if (c < nch && hh >= 0 && hh < H && ww >= 0 && ww < W) {
          u32x4 o;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            float lo = sp_lo(v[m][e]), hi = sp_hi(v[m][e]);
            if constexpr (ACT == ACT_BNRELU) {
              lo = fmaf(lo, sc[2 * e], sh[2 * e]);
              hi = fmaf(hi, sc[2 * e + 1], sh[2 * e + 1]);
            }
            o[e] = sp_pack(fmaxf(lo, 0.f), fmaxf(hi, 0.f));
          }
          sp_wr128(slot + c * 16, o);
        }
      }
      sp_barrier();
    }

    // depthwise 3x3: 5 pixels x 2 channels per lane -> D tile
    char* dx = sx[j & 1];
    {
      float tp[9][2];
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        tp[t][0] = stap[t][s * 32 + 2 * cl];
        tp[t][1] = stap[t][s * 32 + 2 * cl + 1];
      }
      unsigned u[3][SP_SEG + 2];
#pragma unroll
      for (int ky = 0; ky < 3; ++ky)
#pragma unroll
        for (int k = 0; k < SP_SEG + 2; ++k) u[ky][k] = sp_rd32(slot + ky * rowb + wcol[k]);
      sp_lgkm0();
#pragma unroll
      for (int jj = 0; jj < SP_SEG; ++jj) {
        float o[2];
#pragma unroll
        for (int e = 0; e < 2; ++e) {
          float acc_d = 0.f;
#pragma unroll
          for (int ky = 0; ky < 3; ++ky)
#pragma unroll
            for (int kx = 0; kx < 3; ++kx) {
              const unsigned uu = u[ky][jj + kx];
              acc_d = fmaf(e ? sp_hi(uu) : sp_lo(uu), tp[ky * 3 + kx][e], acc_d);
            }
          o[e] = acc_d;
        }
        const int px = x0 + jj;
        if (px < SP_PXB)
          *reinterpret_cast<unsigned*>(dx + px * SP_XP + cl * 4) = px < W ? sp_pack(o[0], o[1]) : 0u;
      }
    }
    sp_barrier();   // D tile complete

    // pointwise: acc[b] += W[16w + .][slice] x D[16b + .][slice]
    {
      const bf16x8 bw = *reinterpret_cast<const bf16x8*>(sw + (w * 16 + fr) * SP_WP + (s * 32 + fg * 8) * 2);
#pragma unroll
      for (int b = 0; b < 10; ++b) {
        const bf16x8 ad = *reinterpret_cast<const bf16x8*>(dx + (b * 16 + fr) * SP_XP + fg * 16);
        acc[b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bw, ad, acc[b], 0, 0, 0);
      }
    }
    // the D slice -> HBM (2 buffer stores per lane, out-of-range lanes dropped)
    const long prow = ((long)n * H + h) * W;
#pragma unroll
    for (int m = 0; m < 2; ++m) {
      const int c = tid + 512 * m;
      const int px = c >> 2, q = c & 3;
      const bool ok = px < W;
      const uint4 v = *reinterpret_cast<const uint4*>(dx + min(px, SP_PXB - 1) * SP_XP + q * 16);
      const unsigned off = ok ? (unsigned)(((prow + px) * CIN + s * 32 + q * 8) * 2) : SP_OOB;
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(i32x4, v), rD, (int)off, 0, 0);
    }
    int st = 2;
    if (s == S - 1) {   // the tile's Y row: 10 stores of 4 channels per lane, then the BN sums
#pragma unroll
      for (int b = 0; b < 10; ++b) {
        const int px = b * 16 + fr;
        float f[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) f[r] = (float)(bf16)acc[b][r];
        const unsigned lo = sp_pack(f[0], f[1]), hi = sp_pack(f[2], f[3]);
        const unsigned off = px < W ? (unsigned)(((prow + px) * SP_CO + w * 16 + 4 * fg) * 2) : SP_OOB;
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(i32x2, make_uint2(lo, hi)), rY, (int)off, 0, 0);
#pragma unroll
        for (int r = 0; r < 4; ++r) {   // (pixels past W hold zero: D rows past W are zero)
          s1[r] += f[r];
          s2[r] = fmaf(f[r], f[r], s2[r]);
        }
        acc[b] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
      st += 10;
    }
    st_prev2 = st_prev1;
    st_prev1 = st;
  }
  // BN partial row of this workgroup: reduce the 16 pixel lanes of each channel group
  if (a.part) {
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) {
        s1[r] += __shfl_xor(s1[r], o, 64);
        s2[r] += __shfl_xor(s2[r], o, 64);
      }
    if (fr == 0) {
      float* p = a.part + (long)blockIdx.x * 2 * SP_CO + w * 16 + 4 * fg;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        p[r] = s1[r];
        p[SP_CO + r] = s2[r];
      }
    }
  }
}

int sp_cus() {
  static const int v = [] {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      n = 0;
    return n > 0 ? n : 256;
  }();
  return v;
}

}  // namespace

extern "C" {

// partial-sum rows xcp_sep_fwd writes (one per workgroup); 0: the shape is not supported
int xcp_sep_fwd_parts(int dtype, int N, int H, int W, int CIN, int COUT) {
  if (dtype != XCP_BF16 || COUT != SP_CO || (CIN != 64 && CIN != 128) || W < 1 || W > SP_WMAX || N <= 0 || H <= 0)
    return 0;
  const long pix = (long)N * H * W;
  if (pix * CIN * 2 > 0x7fffffffL || pix * SP_CO * 2 > 0x7fffffffL) return 0;   // 32-bit buffer offsets
  const long tiles = (long)N * H;
  return (int)(tiles < sp_cus() ? tiles : sp_cus());
}

int xcp_sep_fwd(int dtype, int act, const void* X, const float* scale, const float* shift, const float* dwt, const void* pw,
                void* D, void* Y, float* part, int N, int H, int W, int CIN, int COUT, hipStream_t stream) {
  const int grid = xcp_sep_fwd_parts(dtype, N, H, W, CIN, COUT);
  if (grid <= 0) return XCP_EUNSUPPORTED;
  if (act < ACT_NONE || act > ACT_BNRELU || (act == ACT_BNRELU && (!scale || !shift))) return XCP_EINVAL;
  SepArgs a{(const bf16*)X, scale, shift, dwt, (const bf16*)pw, (bf16*)D, (bf16*)Y, part, N, H, W};
#define SP_LAUNCH(A, C) hipLaunchKernelGGL((sep_fwd_kernel<A, C>), dim3(grid), dim3(512), 0, stream, a)
  if (CIN == 64) {
    if (act == ACT_NONE) SP_LAUNCH(ACT_NONE, 64);
    else if (act == ACT_RELU) SP_LAUNCH(ACT_RELU, 64);
    else SP_LAUNCH(ACT_BNRELU, 64);
  } else {
    if (act == ACT_NONE) SP_LAUNCH(ACT_NONE, 128);
    else if (act == ACT_RELU) SP_LAUNCH(ACT_RELU, 128);
    else SP_LAUNCH(ACT_BNRELU, 128);
  }
#undef SP_LAUNCH
  return (int)hipGetLastError();
}

}  // extern "C"
