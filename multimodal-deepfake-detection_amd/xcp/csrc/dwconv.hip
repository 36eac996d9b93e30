// Depthwise 3x3 convolution (stride 1, pad 1, no bias), NHWC, forward and fused
// backward (dgrad + wgrad + activation mask + residual / skip-gradient adds +
// the BatchNorm-backward partial sums of the preceding BN).
//
// Reference op: SeparableConv2d.conv1 = nn.Conv2d(C, C, 3, 1, 1, groups=C,
// bias=False) (Xception.py:41, called at :45), always preceded in the
// backbone by a ReLU and usually by the previous BatchNorm (Block.rep,
// Xception.py:61-87).  That input transform is applied when the tile is staged:
//   ACT_NONE   : a = x                          (block1's first rep, Xception.py:80-81; conv3)
//   ACT_RELU   : a = max(x, 0)                  (first rep of blocks 2-12, :83)
//   ACT_BNRELU : a = max(x*scale[c]+shift[c], 0) (BN of the previous rep + ReLU)
//
// HBM-bound.  One workgroup = one spatial tile (TH x TW outputs) of one image for
// one 64-byte channel slice (32 bf16 / 16 fp32 channels).  The (TH+2) x
// (nseg*SEGL+2) halo of the input (and of dY in the backward) is staged into LDS
// in the storage type with 16-byte loads, all issued before the first is consumed,
// the activation applied once at staging.  Each lane then owns one dword of
// channels (2 bf16 / 1 fp32) and computes SEGL outputs of a row segment from a
// fully unrolled 3 x (SEGL+2) register window.  FWD_MAXPX (halo pixels per staged
// tile) trades halo re-reads against workgroups per CU (512: 5 workgroups per CU).
#include "common.h"
#include <stdlib.h>

namespace {

constexpr int SLICE = 64;     // bytes of channels per pixel per workgroup
constexpr int NW = 16;        // row workers per workgroup (256 threads = 16 workers x 16 dword lanes)
constexpr int SEGL = 5;       // output pixels per row segment

constexpr int FWD_MAXPX = 512;   // halo pixels per staged forward tile (29.5 KB of LDS at 19x19)

// Tile of TH x TW outputs; the LDS tile is (TH+2) x (nseg*SEGL+2) so every
// segment is exactly SEGL wide (columns past TW / W are computed, never stored).
struct TileGeo {
  int TH, TW, HP, WP, nth, ntw, nseg;
};

inline TileGeo tile_geo(int H, int W, int maxpx, int segl = SEGL) {
  TileGeo g;
  g.ntw = (W + 39) / 40;
  g.TW = (W + g.ntw - 1) / g.ntw;
  g.nseg = (g.TW + segl - 1) / segl;
  g.WP = g.nseg * segl + 2;
  int thmax = maxpx / g.WP - 2;
  if (thmax < 1) thmax = 1;
  g.nth = (H + thmax - 1) / thmax;
  g.TH = (H + g.nth - 1) / g.nth;
  g.HP = g.TH + 2;
  return g;
}

template <typename T> struct DT;
template <> struct DT<bf16> { static constexpr int EPT = 2; };
template <> struct DT<float> { static constexpr int EPT = 1; };

// dword <-> EPT floats
XCP_DEV void unpack(unsigned u, float* v, bf16*) {
  v[0] = __uint_as_float(u << 16);
  v[1] = __uint_as_float(u & 0xffff0000u);
}
XCP_DEV void unpack(unsigned u, float* v, float*) { v[0] = __uint_as_float(u); }
XCP_DEV unsigned pack(const float* v, bf16*) { return pk_bf16(v[0], v[1]); }   // hardware RNE conversion
XCP_DEV unsigned pack(const float* v, float*) { return __float_as_uint(v[0]); }

template <int ACT>
XCP_DEV float act1(float x, float s, float t) {
  if constexpr (ACT == ACT_RELU) return fmaxf(x, 0.f);
  else if constexpr (ACT == ACT_BNRELU) return fmaxf(fmaf(x, s, t), 0.f);
  else return x;
}

// Stage the halo of tensor `src` (pixel rows of C channels) into LDS `dst`
// ([HP*WP][SLICE bytes]); with TRANSFORM the activation is applied.  All global
// loads of a thread are issued before any is consumed (unconditional loads from a
// clamped address, zero-selected afterwards).
typedef int dwi2 __attribute__((ext_vector_type(2)));
constexpr unsigned DW_BUF_OOB = 0x80000000u;     // >= num_records: the access is dropped, a load returns zeros
constexpr int DW_BUF_RECORDS = 0x7fffffff;
constexpr int DW_BUF_DWORD3 = 0x00020000;        // gfx9 raw buffer descriptor word 3

template <typename T, int ACT, bool TRANSFORM, int MAXPX, int FS = SLICE>
XCP_DEV void stage(const T* __restrict__ src, char* dst, const TileGeo& g, long nbase, int th0, int tw0, int H, int W,
                   int C, int c0, const float* scale, const float* shift) {
  constexpr int EPC = 16 / (int)sizeof(T);   // elements per 16-B chunk
  constexpr int CPP = FS / 16;               // chunks per pixel slice
  constexpr int MAXIT = MAXPX * CPP / 256;
  const int total = g.HP * g.WP * CPP;
  static_assert(256 % CPP == 0, "a thread's chunk column must be fixed");
  // this thread always stages the same 16-B channel chunk: fetch its BN affine once
  float sc[EPC], sh[EPC];
  if constexpr (TRANSFORM && ACT == ACT_BNRELU) {
    const int cq = min(c0 + (int)(threadIdx.x % CPP) * EPC, C - EPC);
    VecIO<float, EPC>::load(scale + cq, sc);
    VecIO<float, EPC>::load(shift + cq, sh);
  }
  // Chunk k of this thread is tile pixel p = tid / CPP + k * (256 / CPP), channel chunk tid % CPP: its
  // (row, column) in the padded tile and its byte offset in the frame advance incrementally (a runtime
  // division and a 64-bit address product per chunk were most of this loop's VALU cycles), and the loads
  // go through a buffer resource on the frame, 32-bit offsets (frames are far below 2 GB).
  constexpr int PSTEP = 256 / CPP;
  const int q = threadIdx.x % CPP, c = c0 + q * EPC;
  const int p0 = threadIdx.x / CPP;
  int hy = p0 / g.WP, hx = p0 - hy * g.WP;
  const int dhy = PSTEP / g.WP, dhx = PSTEP - dhy * g.WP;
  const int rowb = W * C * (int)sizeof(T), pixb = C * (int)sizeof(T);
  int boff = (th0 - 1 + hy) * rowb + (tw0 - 1 + hx) * pixb + c * (int)sizeof(T);
  const int stepb = dhy * rowb + dhx * pixb, wrapb = rowb - g.WP * pixb;
  const __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<T*>(src + nbase * C), (short)0, DW_BUF_RECORDS, DW_BUF_DWORD3);
  uint4 v[MAXIT];
  bool ok[MAXIT];
#pragma unroll
  for (int k = 0; k < MAXIT; ++k) {
    const int i = threadIdx.x + 256 * k;
    const int h = th0 - 1 + hy, w = tw0 - 1 + hx;
    ok[k] = i < total && h >= 0 && h < H && w >= 0 && w < W && c < C;
    v[k] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, ok[k] ? boff : (int)DW_BUF_OOB, 0, 0));
    hx += dhx;
    hy += dhy;
    boff += stepb;
    if (hx >= g.WP) {
      hx -= g.WP;
      ++hy;
      boff += wrapb;
    }
  }
#pragma unroll
  for (int k = 0; k < MAXIT; ++k) {
    const int i = threadIdx.x + 256 * k;
    if (i >= total) break;
    const int p = i / CPP;
    uint4 u = v[k];   // (zero where !ok: the out-of-range load returns zeros)
    if constexpr (TRANSFORM && ACT != ACT_NONE) {
      if (ok[k]) {
        float f[EPC];
        VecIO<T, EPC>::load(reinterpret_cast<const T*>(&u), f);
        typedef float p2 __attribute__((ext_vector_type(2)));
#pragma unroll
        for (int j = 0; j < EPC; j += 2) {   // packed pairs (v_pk_fma_f32 / v_pk_max_f32)
          p2 v = p2{f[j], f[j + 1]};
          if constexpr (ACT == ACT_BNRELU) v = __builtin_elementwise_fma(v, p2{sc[j], sc[j + 1]}, p2{sh[j], sh[j + 1]});
          v = __builtin_elementwise_max(v, p2(0.f));
          f[j] = v[0];
          f[j + 1] = v[1];
        }
        VecIO<T, EPC>::store(reinterpret_cast<T*>(&u), f);
      }
    }
    *reinterpret_cast<uint4*>(dst + p * FS + q * 16) = u;
  }
}

XCP_DEV int block_coords(int ngroups, const TileGeo& g, int& grp, int& n, int& th0, int& tw0) {
  const int id = xcd_remap(blockIdx.x, gridDim.x);
  grp = id % ngroups;
  const int sp = id / ngroups;
  const int ntiles = g.nth * g.ntw;
  const int tile = sp % ntiles;
  n = sp / ntiles;
  th0 = (tile / g.ntw) * g.TH;
  tw0 = (tile % g.ntw) * g.TW;
  return sp;
}

struct DwArgs {
  const void* X;        // [N,H,W,C] raw input (pre-transform)
  void* Y;              // [N,H,W,C] output
  const float* Wt;      // [9][C] taps (tap = ky*3+kx)
  const float* scale;   // [C] (ACT_BNRELU)
  const float* shift;   // [C]
  int N, H, W, C, ngroups;
  TileGeo g;
};

// FS: bytes of channels per pixel per workgroup (64, or 128 when the channel pitch is a
// multiple of 128 B, so each pixel slice is one whole cache line)
template <typename T, int ACT, int MAXPX, int FS>
__global__ __launch_bounds__(256) void dw_fwd_kernel(DwArgs a) {
  constexpr int LANES = FS / 4;           // dword lanes per row worker
  constexpr int NWK = 256 / LANES;        // row workers per workgroup
  constexpr int EPT = DT<T>::EPT;
  constexpr int CPG = FS / (int)sizeof(T);      // channels per group
  __shared__ __attribute__((aligned(16))) char sA[MAXPX * FS];
  const TileGeo& g = a.g;
  int grp, n, th0, tw0;
  block_coords(a.ngroups, g, grp, n, th0, tw0);
  const int c0 = grp * CPG;
  const long nbase = (long)n * a.H * a.W;
  const int cl = threadIdx.x % LANES, wk = threadIdx.x / LANES;
  const int c = c0 + cl * EPT;
  const int cc = c < a.C ? c : a.C - EPT;
  float wt[9][EPT];
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int e = 0; e < EPT; ++e) wt[t][e] = a.Wt[(long)t * a.C + cc + e];
  stage<T, ACT, true, MAXPX, FS>(reinterpret_cast<const T*>(a.X), sA, g, nbase, th0, tw0, a.H, a.W, a.C, c0, a.scale,
                             a.shift);
  __syncthreads();
  if (c >= a.C) return;
  // stores and item walk as dw_fwd_w2_kernel (buffer resource on the frame, dropped out-of-range stores)
  T* Y = reinterpret_cast<T*>(a.Y);
  const __amdgpu_buffer_rsrc_t rY =
      __builtin_amdgcn_make_buffer_rsrc(Y + nbase * a.C, (short)0, DW_BUF_RECORDS, DW_BUF_DWORD3);
  const int items = g.TH * g.nseg;
  const char* lbase = sA + cl * 4;
  const int xlim = min(g.TW, a.W - tw0);
  const int nseg = g.nseg, dr = NWK / nseg, ds = NWK - dr * nseg;
  int r = wk / nseg, sg = wk - r * nseg;
  for (int it = wk; it < items; it += NWK) {
    const int oh = th0 + r;
    const int x0 = sg * SEGL;
    if (oh < a.H) {
      const char* base = lbase + (r * g.WP + x0) * FS;
      float win[3][SEGL + 2][EPT];
#pragma unroll
      for (int ky = 0; ky < 3; ++ky)
#pragma unroll
        for (int k = 0; k < SEGL + 2; ++k)
          unpack(*reinterpret_cast<const unsigned*>(base + (ky * g.WP + k) * FS), win[ky][k], (T*)nullptr);
      const int off = ((oh * a.W + tw0 + x0) * a.C + c) * (int)sizeof(T);
#pragma unroll
      for (int j = 0; j < SEGL; ++j) {
        float o[EPT];
        // (one fma chain per channel in (ky, kx) order: the summation order the bf16 parity
        // tests were pinned with; a per-row split into packed pairs measured only ~3 % faster)
#pragma unroll
        for (int e = 0; e < EPT; ++e) {
          float s = 0.f;
#pragma unroll
          for (int ky = 0; ky < 3; ++ky)
#pragma unroll
            for (int kx = 0; kx < 3; ++kx) s = fmaf(win[ky][j + kx][e], wt[ky * 3 + kx][e], s);
          o[e] = s;
        }
        __builtin_amdgcn_raw_buffer_store_b32((int)pack(o, (T*)nullptr), rY,
                                              x0 + j < xlim ? off + j * a.C * (int)sizeof(T) : (int)DW_BUF_OOB, 0, 0);
      }
    }
    sg += ds;
    r += dr;
    if (sg >= nseg) {
      sg -= nseg;
      ++r;
    }
  }
}

// The same forward with two channel dwords (4 bf16 channels) per lane: 8 lanes per 64-B pixel
// slice, 32 row workers of SG-pixel segments, one 8-B store per output pixel and lane (half the
// store instructions of dw_fwd_kernel's 4-B stores); the per-channel fma chain is the same, so
// the outputs are bitwise those of dw_fwd_kernel.
template <int ACT, int MAXPX, int SG>
__global__ __launch_bounds__(256) void dw_fwd_w2_kernel(DwArgs a) {
  constexpr int FS = SLICE, LANES = FS / 8, NWK = 256 / LANES, CPL = 4;
  __shared__ __attribute__((aligned(16))) char sA[MAXPX * FS];
  const TileGeo& g = a.g;
  int grp, n, th0, tw0;
  block_coords(a.ngroups, g, grp, n, th0, tw0);
  const int c0 = grp * (FS / 2);
  const long nbase = (long)n * a.H * a.W;
  const int cl = threadIdx.x % LANES, wk = threadIdx.x / LANES;
  const int c = c0 + cl * CPL;
  const int cc = c < a.C ? c : a.C - CPL;
  float wt[9][CPL];
#pragma unroll
  for (int t = 0; t < 9; ++t) VecIO<float, CPL>::load(a.Wt + (long)t * a.C + cc, wt[t]);
  stage<bf16, ACT, true, MAXPX, FS>(reinterpret_cast<const bf16*>(a.X), sA, g, nbase, th0, tw0, a.H, a.W, a.C, c0, a.scale,
                                    a.shift);
  __syncthreads();
  if (c >= a.C) return;
  // Y through a buffer resource on the frame: 32-bit byte offsets (a frame is far below 2 GB), and the
  // pixels past the tile or the image get an out-of-range offset, so the store is dropped instead of
  // branched around; the item walk advances (row, segment) incrementally.  (The 64-bit per-pixel
  // address products and the per-item division were a fifth of the loop's VALU cycles.)
  bf16* Y = reinterpret_cast<bf16*>(a.Y);
  const __amdgpu_buffer_rsrc_t rY =
      __builtin_amdgcn_make_buffer_rsrc(Y + nbase * a.C, (short)0, DW_BUF_RECORDS, DW_BUF_DWORD3);
  const int items = g.TH * g.nseg;
  const char* lbase = sA + cl * 8;
  const int xlim = min(g.TW, a.W - tw0);                 // tile columns inside the image
  const int nseg = g.nseg, dr = NWK / nseg, ds = NWK - dr * nseg;
  int r = wk / nseg, sg = wk - r * nseg;
  for (int it = wk; it < items; it += NWK) {
    const int oh = th0 + r;
    const int x0 = sg * SG;
    if (oh < a.H) {
      const char* base = lbase + (r * g.WP + x0) * FS;
      float win[3][SG + 2][CPL];
#pragma unroll
      for (int ky = 0; ky < 3; ++ky)
#pragma unroll
        for (int k = 0; k < SG + 2; ++k) {
          const uint2 u = *reinterpret_cast<const uint2*>(base + (ky * g.WP + k) * FS);
          unpack(u.x, win[ky][k], (bf16*)nullptr);
          unpack(u.y, win[ky][k] + 2, (bf16*)nullptr);
        }
      const int off = ((oh * a.W + tw0 + x0) * a.C + c) * 2;
#pragma unroll
      for (int j = 0; j < SG; ++j) {
        float o[CPL];
#pragma unroll
        for (int e = 0; e < CPL; ++e) {
          float s = 0.f;
#pragma unroll
          for (int ky = 0; ky < 3; ++ky)
#pragma unroll
            for (int kx = 0; kx < 3; ++kx) s = fmaf(win[ky][j + kx][e], wt[ky * 3 + kx][e], s);
          o[e] = s;
        }
        const uint2 v = make_uint2(pack(o, (bf16*)nullptr), pack(o + 2, (bf16*)nullptr));
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(dwi2, v), rY,
                                              x0 + j < xlim ? off + j * a.C * 2 : (int)DW_BUF_OOB, 0, 0);
      }
    }
    sg += ds;
    r += dr;
    if (sg >= nseg) {
      sg -= nseg;
      ++r;
    }
  }
}

// bf16 64-B-slice forwards run dw_fwd_w2_kernel with 5-pixel segments by default: 67 -> 64.5 us
// at 19^2 x 736, 262 -> 246 at 37^2, 766 -> 733 at 147^2 x 128, bitwise-equal outputs
// (tools/kbench.py dwshapes fingerprints, profiles/r03_dw_fwd_w2_ab.txt).  XCP_DW_FWD_W2=0 selects
// dw_fwd_kernel, =4 4-pixel segments (A/B).
int dw_fwd_w2() {
  static const int v = [] {
    const char* e = getenv("XCP_DW_FWD_W2");
    const int k = e ? atoi(e) : 5;
    return k == 4 || k == 5 ? k : 0;
  }();
  return v;
}

// ---------------------------------------------------------------------------------
// Fused backward.  Per pixel p:
//   dA[p]   = sum_tap dY[p - off(tap)] * w[tap]          (transposed 3x3)
//   dX[p]   = act'(p) * dA[p] + dRes[p] + (p at stride-multiple (h,w) ? dSkip[p/s] : 0)
//   dW[tap] += dY[p] * a[p + off(tap)]                   (workgroup partial -> slab)
// act'(p) = (a[p] > 0) for ACT_RELU / ACT_BNRELU, 1 for ACT_NONE.  For ACT_BNRELU
// dX is the gradient w.r.t. the preceding BN's output z; when bnpart is given the
// workgroup also emits that BN's backward partial sums (sum dz, sum dz*zhat) with
// zhat = (x - mean) * invstd, taken over the stored (rounded) dz.
struct DwBwdArgs {
  const void* dY;
  const void* X;
  const float* Wt;
  const float* scale;
  const float* shift;
  const void* dRes;
  const void* dSkip;
  int sOH, sOW, sS;
  int skip_pre;           // 1: the skip term is a gradient of the same activation (added before the
                          // activation mask and the BN partial sums), 0: added after them
  void* dX;
  float* dWpart;          // [P][C][9]
  float* bnpart;          // [P][2][C] or null
  const void* Yb;         // with dRes: the sums are those of the BN whose output gradient is the final dX
                          // (after the residual add), zhat = (Yb - mean) * invstd (xcp_dw_bwd_resbn)
  const float* bmean;
  const float* binvstd;
  int N, H, W, C, ngroups;
  int nbands, bandH;      // row bands per frame (one wave walks rows [band*bandH, +bandH))
  int xcd;                // 1: consecutive workgroups of the walk on one XCD (xcd_remap)
};

template <typename T, int P, int FS>
int launch_fwd(int act, const DwArgs& a, hipStream_t st) {
  const int blocks = a.N * a.g.nth * a.g.ntw * a.ngroups;
  if (act == ACT_NONE) hipLaunchKernelGGL((dw_fwd_kernel<T, ACT_NONE, P, FS>), dim3(blocks), dim3(256), 0, st, a);
  else if (act == ACT_RELU) hipLaunchKernelGGL((dw_fwd_kernel<T, ACT_RELU, P, FS>), dim3(blocks), dim3(256), 0, st, a);
  else hipLaunchKernelGGL((dw_fwd_kernel<T, ACT_BNRELU, P, FS>), dim3(blocks), dim3(256), 0, st, a);
  return (int)hipGetLastError();
}

inline int ngroups_for(int C, int dtype, int slice = SLICE) {
  const int cpg = slice / (dtype == XCP_BF16 ? 2 : 4);
  return (C + cpg - 1) / cpg;
}

// Forward slice bytes: 128 (whole cache lines, half the workgroups, twice the work each) for
// small frames whose halo tile fits FWD_MAXPX128 pixels and whose pixel rows start on a line;
// else 64.  Measured (tools/kbench.py dwshapes, 256 frames): 10^2 x 1536 / 2048 47.7 -> 36.7 /
// 69.2 -> 52.6 us; at 19^2 and larger 128-B slices were 0-5 % slower (3 tiles per frame).
constexpr int FWD_MAXPX128 = 256;   // halo pixels per staged 128-B-slice tile (32 KB)
inline int fwd_slice_bytes(int C, int esz, int H, int W) {
  return (C * esz) % 128 == 0 && (H + 2) * (W + 2) <= FWD_MAXPX128 ? 128 : 64;
}


// =================================================================================
// Backward: one WAVE owns one channel slice (64 B: 32 bf16 / 16 fp32 channels) of one
// frame over RCOLS = 20 output columns and walks down all H rows: lane (cl, s) =
// (lane & 15, lane >> 4) holds one channel dword (2 bf16 -> float2, packed
// v_pk_fma_f32 math) for the 5 output columns 5s .. 5s+4 of the wave's column range,
// with rolling 3-row register windows.  dW / BN partial sums are reduced over the 4
// lane segments with cross-lane shuffles and written once per (frame, column group):
// P = N * ceil(W / 20).
constexpr int RS = 5, RNS = 4, RCOLS = RS * RNS;
typedef float rf2 __attribute__((ext_vector_type(2)));

template <typename T> struct RV;
template <> struct RV<bf16> {
  typedef rf2 V;
  static constexpr int EPT = 2;
  static XCP_DEV V unpack(unsigned u) { return V{__uint_as_float(u << 16), __uint_as_float(u & 0xffff0000u)}; }
  static XCP_DEV unsigned pack(V v) { return pk_bf16(v[0], v[1]); }
  static XCP_DEV V load(const float* p) { return V{p[0], p[1]}; }
  static XCP_DEV float get(V v, int e) { return v[e]; }
};
template <> struct RV<float> {
  typedef float V;
  static constexpr int EPT = 1;
  static XCP_DEV V unpack(unsigned u) { return __uint_as_float(u); }
  static XCP_DEV unsigned pack(V v) { return __float_as_uint(v); }
  static XCP_DEV V load(const float* p) { return p[0]; }
  static XCP_DEV float get(V v, int) { return v; }
};

template <typename V> XCP_DEV V vfma(V a, V b, V c) { return __builtin_elementwise_fma(a, b, c); }
template <typename V> XCP_DEV V vmax0(V a) { return __builtin_elementwise_max(a, V(0.f)); }

struct RowMap {
  int n, cg, grp, unit, band;
  bool live;
};
XCP_DEV RowMap row_map(int N, int ncg, int ngroups, int nbands = 1, bool xcd = false) {
  RowMap m;
  // xcd: the workgroups holding consecutive channel slices of a pixel row run on one XCD, so the
  // 128-B lines two of them share (every odd pixel of a 1,472-B row starts mid-line) are fetched
  // into one L2 instead of two
  const int wg = xcd ? xcd_remap(blockIdx.x, gridDim.x) : blockIdx.x;
  const int gw = __builtin_amdgcn_readfirstlane(wg * 4 + (threadIdx.x >> 6));
  m.live = gw < N * ncg * nbands * ngroups;
  m.grp = gw % ngroups;
  m.unit = gw / ngroups;   // (frame, column group, row band): the partial-sum row
  m.band = m.unit % nbands;
  const int fc = m.unit / nbands;
  m.cg = fc % ncg;
  m.n = fc / ncg;
  return m;
}

// =================================================================================
// LDS-staged row walk: every HBM access is 16 B per lane: each input row of the
// wave (22 pixels x 64 B, 1408 B) is brought into a per-wave LDS ring by LDS-DMA
// (global_load_lds, out-of-range pixels and rows from a zero line), lanes read their
// 7-column windows from LDS, and each output row is staged in LDS and written with
// 16-B stores (a register-load row walk was limited by the texture address path at one
// VMEM lane-op per 2 channels; here it is one per 8).
// Waves are independent (no barriers).  Every step issues the same number of VMEM
// instructions (masked lanes read the zero line / write a sink), so the per-wave
// vmcnt counts are static; VMEM operations retire in issue order.
constexpr int LROW = (RCOLS + 2) * SLICE;   // 1408 B: one staged row of one tensor
__device__ __attribute__((aligned(64))) uint4 g_dzero[4];
__device__ __attribute__((aligned(64))) uint4 g_dsink[64];

// s_waitcnt vmcnt(N) as a real S_WAITCNT (gfx9 encoding: vmcnt[3:0] | expcnt[6:4] |
// lgkmcnt[11:8] | vmcnt_hi[15:14]), so the compiler's own wait insertion sees it
template <int N>
XCP_DEV void vmwait() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 15) | (0x7 << 4) | (0xF << 8) | ((N >> 4) << 14));
}

// Per-lane element offsets, within one frame row, of the two 16-B chunks a lane moves in
// stage_row / store_row (-1: the zero line / the sink).  Computed once per wave, so a row
// step's addresses are one scalar row offset plus these (no per-step 64-bit multiplies).
struct RowLanes {
  int off[2];
};

// load side: pixels x0w-1 .. x0w+20 of the 64-B slice at channel c0
template <typename T>
XCP_DEV RowLanes row_lanes_load(int W, int C, int x0w, int c0, int lane) {
  constexpr int EPC = 16 / (int)sizeof(T);
  RowLanes r;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int ch = i * 64 + lane;            // chunk: pixel ch >> 2, 16-B part ch & 3
    const int col = x0w - 1 + (ch >> 2);
    const int c = c0 + (ch & 3) * EPC;
    r.off[i] = (col >= 0 && col < W && c < C) ? col * C + c : -1;
  }
  return r;
}

// store side: pixels x0w .. x0w+19
template <typename T>
XCP_DEV RowLanes row_lanes_store(int W, int C, int x0w, int c0, int lane) {
  constexpr int EPC = 16 / (int)sizeof(T);
  RowLanes r;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int ch = i * 64 + lane;
    const int p = ch >> 2, col = x0w + p;
    const int c = c0 + (ch & 3) * EPC;
    r.off[i] = (p < RCOLS && col < W && c < C) ? col * C + c : -1;
  }
  return r;
}

// Stage pixels x0w-1 .. x0w+20 (64-B slice at channel c0) of row h of a frame into
// dst (LDS, 1408 B) with two LDS-DMA instructions (88 lanes of 16 B).
// The frame is a buffer resource (SGPRs): the row's offset is scalar, the lane's part fixed, and
// rows past H / pixels outside the frame get an out-of-range offset (the DMA writes zeros) -- no
// 64-bit address or select of a zero-line pointer per instruction.
template <typename T>
XCP_DEV void stage_row(__amdgpu_buffer_rsrc_t frame, int h, int H, int W, int C, const RowLanes& rl, char* dst, int lane) {
  // (rows past H: a base at the out-of-range bound, so every lane's offset is out of range without a
  // branch on the row)
  const unsigned rowb = h < H ? (unsigned)(h * W * C * (int)sizeof(T)) : DW_BUF_OOB;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int o = rl.off[i] >= 0 ? (int)(rowb + (unsigned)(rl.off[i] * (int)sizeof(T))) : (int)DW_BUF_OOB;
    if (i == 0 || lane < 24)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(frame, (__attribute__((address_space(3))) void*)(dst + i * 1024), 16, o,
                                               0, 0, 0);
  }
}

// Write the staged output row (20 pixels x 64 B in `stg`) to row h: two 16-B stores
// per lane-slot; lanes without a valid pixel write the sink.  The staging reads are inline asm:
// the staging shares the ring's LDS object, and a compiler-visible read of it would make hipcc
// wait for every LDS-DMA in flight (vmcnt(0): the look-ahead rows) before the stores.
typedef unsigned dwu4 __attribute__((ext_vector_type(4)));
template <typename T>
XCP_DEV void store_row(T* frame, int h, int W, int C, const RowLanes& rl, const char* stg, int lane) {
  T* row = frame + (long)h * W * C;
  dwu4 v[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int ch = i * 64 + lane;
    asm volatile("ds_read_b128 %0, %1"
                 : "=v"(v[i])
                 : "v"((unsigned)(size_t)(const __attribute__((address_space(3))) char*)(stg + min(ch, 4 * RCOLS - 1) * 16))
                 : "memory");
  }
  asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(v[0]), "+v"(v[1]) : : "memory");
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    uint4* dstp = rl.off[i] >= 0 ? reinterpret_cast<uint4*>(row + rl.off[i]) : g_dsink + lane;
    *dstp = make_uint4(v[i][0], v[i][1], v[i][2], v[i][3]);
  }
}

// LDS reads of the DMA ring by inline asm (XCP_DW_BWD_ASM=1): while the output staging was a second
// __shared__ object, a plain C++ read of the ring made hipcc drain every outstanding vector-memory
// operation first (s_waitcnt vmcnt(0)), right after a step had issued the look-ahead rows; the asm
// reads avoided that.  With one LDS object the plain reads carry no such wait
// (test_dma_pipelines_not_drained_by_compiler_waits).  The counted vmwait at the top of a step is what
// orders the ring; ring_fence() retires the asm reads before their values are used (pinned through
// "+v" operands, so no use is scheduled ahead of the wait).
XCP_DEV unsigned ring_u32(const char* p) {
  unsigned v;
  asm volatile("ds_read_b32 %0, %1" : "=v"(v) : "v"((unsigned)(size_t)(const __attribute__((address_space(3))) char*)(p))
               : "memory");
  return v;
}
template <int N>
XCP_DEV void ring_fence(unsigned (&v)[N]) {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
  for (int i = 0; i < N; ++i) asm volatile("" : "+v"(v[i]));
}
XCP_DEV void ring_fence1(unsigned& v) {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  asm volatile("" : "+v"(v));
}

// Without a residual input (ROLL = false) the three dY rows a step needs (h-1, h, h+1) are read
// from the LDS ring one row at a time and consumed at once (dgrad and wgrad FMAs of that row), so
// only one 7-column window is live instead of three rolling ones: 177 -> 140-152 VGPRs, three
// waves per SIMD instead of two (the dY ring keeps BD + 3 slots: rows h-1 .. h+1 being read, h+2
// landed, h+3 staged).  With the residual (ROLL = true) the extra ring slots would cost a
// workgroup per CU (LDS), so the rolling register windows stay: measured 125.2 vs 138.6 us
// without, 148.1 vs 142.3 us with the residual at 19^2 x 736 (profiles/r03_dwb_ab.txt).
// BNRES: the BN partial sums are taken over the final dX against a.Yb (xcp_dw_bwd_resbn; a template
// argument so the other forms carry no conditional loads -- a load behind a runtime branch made hipcc
// drain vmcnt(0) at the branch's join on every row step)
template <typename T, int ACT, bool RES, bool ROLL, int BDV = 2, int MINW = (ROLL ? 2 : 3), bool SKIP = true,
          bool BNRES = false, bool ASMRD = false>
__global__ __launch_bounds__(256, MINW) void dw_bwd_lds_kernel(DwBwdArgs a) {
  typedef RV<T> R;
  typedef typename R::V V;
  constexpr int EPT = R::EPT, CPG = 16 * EPT;
  constexpr int BD = BDV;                                // rows of look-ahead per staged tensor
  constexpr int NS = BD + 1;                             // X / dRes ring slots
  constexpr int NSG = ROLL ? NS : BD + 3;                // dY ring slots
  // one LDS object for the rings and the output staging: with a second object the LDS accesses carry
  // alias scopes, and hipcc then drains every in-flight LDS-DMA (vmcnt(0)) ahead of the first plain
  // ring read of a step, right after the look-ahead row was issued
  constexpr int RING = (NS + NSG + (RES ? NS : 0)) * LROW;
  __shared__ __attribute__((aligned(16))) char sm[4 * RING + 4 * RCOLS * SLICE];
  const int ncg = (a.W + RCOLS - 1) / RCOLS;
  const RowMap mp = row_map(a.N, ncg, a.ngroups, a.nbands, a.xcd != 0);
  if (!mp.live) return;
  // this wave's rows [r0, r1); it reads X rows r0 .. r1-1 and dY rows r0-1 .. r1 (rows past
  // those are staged from the zero line: never read)
  const int r0 = mp.band * a.bandH, r1 = min(a.H, r0 + a.bandH);
  const int hx = r1, hg = min(a.H, r1 + 1);
  const int lane = threadIdx.x & 63, cl = lane & 15, sg = lane >> 4;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);   // (wave-uniform: the DMA's LDS address is M0)
  char* ring = sm + wv * RING;
  char* rx = ring;                  // X rows, slot r % NS
  char* rg = ring + NS * LROW;      // dY rows, slot r % NSG
  char* rres = rg + NSG * LROW;     // dRes rows (RES), slot r % NS
  char* stg = sm + 4 * RING + wv * (RCOLS * SLICE);
  const int c0 = mp.grp * CPG;
  const int c = c0 + cl * EPT;
  const bool cok = c < a.C;
  const int cc = cok ? c : a.C - EPT;
  const int x0w = mp.cg * RCOLS, x0 = x0w + sg * RS;
  const RowLanes rl_ld = row_lanes_load<T>(a.W, a.C, x0w, c0, lane);
  const RowLanes rl_st = row_lanes_store<T>(a.W, a.C, x0w, c0, lane);
  const bool bnsum = a.bnpart != nullptr;
  constexpr bool bnres = RES && BNRES;                  // sums over the final dX against Yb (bnsum implied)
  const bool bnx = bnsum && !bnres;                     // sums over the masked dz against X
  V wt[9], dw[9], sc = V(1.f), sh = V(0.f), bs1 = V(0.f), bs2 = V(0.f), mu = V(0.f), is = V(0.f);
#pragma unroll
  for (int t = 0; t < 9; ++t) {
    wt[t] = R::load(a.Wt + (long)t * a.C + cc);
    dw[t] = V(0.f);
  }
  if constexpr (ACT == ACT_BNRELU) {
    sc = R::load(a.scale + cc);
    sh = R::load(a.shift + cc);
  }
  if (bnsum) {
    mu = R::load(a.bmean + cc);
    is = R::load(a.binvstd + cc);
  }
  unsigned okm = 0;
#pragma unroll
  for (int k = 0; k < RS + 2; ++k) {
    const int col = x0 - 1 + k;
    okm |= (col >= 0 && col < a.W) ? (1u << k) : 0u;
  }
  const long fbase = (long)mp.n * a.H * a.W * a.C;
  auto frame_rsrc = [&](const void* t) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<T*>(reinterpret_cast<const T*>(t) + fbase), (short)0,
                                             DW_BUF_RECORDS, DW_BUF_DWORD3);
  };
  const __amdgpu_buffer_rsrc_t X = frame_rsrc(a.X), G = frame_rsrc(a.dY);
  const __amdgpu_buffer_rsrc_t dRes = frame_rsrc(RES ? a.dRes : a.X);
  const T* dSkip = reinterpret_cast<const T*>(a.dSkip);
  T* dX = reinterpret_cast<T*>(a.dX) + fbase;
  const int lofs = sg * RS * SLICE + cl * 4;
  // ring reads: inline asm retired by fence() (ASMRD), or plain C++ reads (hipcc's own waits; see
  // ring_u32 above and launch_bwd_act for where each form is used)
  auto rd = [&](const char* row, int k) {
    if constexpr (ASMRD) return ring_u32(row + lofs + k * SLICE);
    else return *reinterpret_cast<const unsigned*>(row + lofs + k * SLICE);
  };
  auto fence = [&](auto& v) {
    if constexpr (ASMRD) ring_fence(v);
  };
  auto cvtg = [&](const char* row, V (&gy)[RS + 2]) {
    unsigned u[RS + 2];
#pragma unroll
    for (int k = 0; k < RS + 2; ++k) u[k] = rd(row, k);
    fence(u);
#pragma unroll
    for (int k = 0; k < RS + 2; ++k) gy[k] = R::unpack(u[k]);   // staged zero padding
  };
  auto sx = [&](int r) { return rx + (r % NS) * LROW; };
  auto sgs = [&](int r) { return rg + ((r + NSG) % NSG) * LROW; };   // (r >= -1)
  auto sr = [&](int r) { return rres + (r % NS) * LROW; };
  // VMEM per step h: loads X h+BD, dY h+1+BD (, dRes h+BD) = L, then 2 stores of row h.
  // At step h the rows issued at step h-BD+1 ... are not needed yet; the step-h rows
  // (X h, dY h+1, dRes h) were issued at step h-BD: issued after them are 2 stores
  // + (BD-1) x (L + 2).
  constexpr int L = RES ? 6 : 4;
  auto step = [&](int h, const V (&g0)[RS + 2], const V (&g1)[RS + 2], V (&g2)[RS + 2]) {
    char* sxh = sx(h);
    char* srh = sr(h);
    vmwait<2 + (BD - 1) * (L + 2)>();
    // strided-skip gradient terms of this row: plain loads issued before this step's
    // LDS-DMA, so waiting for them never waits for the prefetch
    const bool skip_row = SKIP && dSkip && (h % a.sS) == 0 && h / a.sS < a.sOH;
    unsigned pskp[RS];
#pragma unroll
    for (int j = 0; j < RS; ++j) pskp[j] = 0u;
    unsigned pyb[RES ? RS : 1];
    if constexpr (RES) {
      if constexpr (bnres) {   // raw values of the BN input at this row's output pixels (clamped column, masked below)
        const T* yrow = reinterpret_cast<const T*>(a.Yb) + fbase + (long)h * a.W * a.C + cc;
#pragma unroll
        for (int j = 0; j < RS; ++j) pyb[j] = *reinterpret_cast<const unsigned*>(yrow + (long)min(x0 + j, a.W - 1) * a.C);
      }
    }
    if constexpr (SKIP) {
      // every step issues the same loads from clamped addresses (masked afterwards): a load behind
      // a runtime branch makes hipcc drain vmcnt(0) where the branch joins, on every row step
      const int srow = min(h / a.sS, max(a.sOH - 1, 0));
#pragma unroll
      for (int j = 0; j < RS; ++j) {
        const int ow = x0 + j;
        const bool ok = skip_row && cok && ow % a.sS == 0 && ow / a.sS < a.sOW && ow < a.W;
        const int scol = min(max(ow, 0) / a.sS, max(a.sOW - 1, 0));
        const T* ptr = dSkip ? dSkip + (((long)mp.n * a.sOH + srow) * a.sOW + scol) * a.C + cc
                             : reinterpret_cast<const T*>(g_dzero);
        const unsigned v = *reinterpret_cast<const unsigned*>(ptr);
        pskp[j] = ok ? v : 0u;
      }
    }
    // activated X row h (slot sxh; zero padded after the activation), raw centre values
    // (at four waves per SIMD the raw centre values are re-read from LDS where the BN sums use them)
    constexpr bool KEEP_XR = MINW < 4;
    V xa[RS + 2];
    unsigned xr[KEEP_XR ? RS : 1];
    unsigned xu[RS + 2];
#pragma unroll
    for (int k = 0; k < RS + 2; ++k) xu[k] = rd(sxh, k);
    fence(xu);
#pragma unroll
    for (int k = 0; k < RS + 2; ++k) {
      const unsigned u = xu[k];
      V v = R::unpack(u);
      if constexpr (ACT == ACT_BNRELU) {
        v = vmax0(vfma(v, sc, sh));
        v = ((okm >> k) & 1) ? v : V(0.f);
      } else if constexpr (ACT == ACT_RELU) {
        v = vmax0(v);
      }
      xa[k] = v;
      if constexpr (KEEP_XR)
        if (k >= 1 && k <= RS) xr[k - 1] = u;
    }
    if constexpr (ROLL) cvtg(sgs(h + 1), g2);   // dY row h+1
    unsigned pres[RS];
    if constexpr (RES) {
#pragma unroll
      for (int j = 0; j < RS; ++j) pres[j] = rd(srh, j + 1);
      fence(pres);
    }
    stage_row<T>(X, h + BD, hx, a.W, a.C, rl_ld, sx(h + BD), lane);          // slot of X row h-1
    stage_row<T>(G, h + 1 + BD, hg, a.W, a.C, rl_ld, sgs(h + 1 + BD), lane);   // slot of dY row h
    if constexpr (RES) stage_row<T>(dRes, h + BD, hx, a.W, a.C, rl_ld, sr(h + BD), lane);
    // dY rows h+1, h, h-1 (ky = 0, 1, 2; row -1 is the zero padding above the frame), one 7-column
    // window at a time; independent accumulation chains: consecutive packed FMAs never depend on
    // each other
    V sj[RS];
#pragma unroll
    for (int j = 0; j < RS; ++j) sj[j] = V(0.f);
    if constexpr (ROLL) {
#pragma unroll
      for (int kx = 0; kx < 3; ++kx)
#pragma unroll
        for (int ky = 0; ky < 3; ++ky)
#pragma unroll
          for (int j = 0; j < RS; ++j)
            sj[j] = vfma((ky == 0 ? g2 : ky == 1 ? g1 : g0)[j + 2 - kx], wt[ky * 3 + kx], sj[j]);
#pragma unroll
      for (int j = 0; j < RS; ++j)
#pragma unroll
        for (int kx = 0; kx < 3; ++kx) {
          dw[kx] = vfma(g2[j + 1], xa[j + kx], dw[kx]);
          dw[3 + kx] = vfma(g1[j + 1], xa[j + kx], dw[3 + kx]);
          dw[6 + kx] = vfma(g0[j + 1], xa[j + kx], dw[6 + kx]);
        }
    } else {
#pragma unroll
      for (int ky = 0; ky < 3; ++ky) {
        V gw[RS + 2];
        cvtg(sgs(h + 1 - ky), gw);
        if (ky == 2 && h == 0) {
#pragma unroll
          for (int k = 0; k < RS + 2; ++k) gw[k] = V(0.f);
        }
#pragma unroll
        for (int kx = 0; kx < 3; ++kx)
#pragma unroll
          for (int j = 0; j < RS; ++j) sj[j] = vfma(gw[j + 2 - kx], wt[ky * 3 + kx], sj[j]);
#pragma unroll
        for (int j = 0; j < RS; ++j)
#pragma unroll
          for (int kx = 0; kx < 3; ++kx) dw[ky * 3 + kx] = vfma(gw[j + 1], xa[j + kx], dw[ky * 3 + kx]);
      }
    }
#pragma unroll
    for (int j = 0; j < RS; ++j) {
      V s = sj[j];
      if (skip_row && a.skip_pre) s += R::unpack(pskp[j]);
      if constexpr (ACT != ACT_NONE) {
        const V ctr = xa[j + 1];
        if constexpr (EPT == 2) {
          s[0] = ctr[0] > 0.f ? s[0] : 0.f;
          s[1] = ctr[1] > 0.f ? s[1] : 0.f;
        } else {
          s = ctr > 0.f ? s : 0.f;
        }
      }
      if (bnx) {
        const bool valid = cok && x0 + j < a.W;
        const V dz = valid ? R::unpack(R::pack(s)) : V(0.f);   // the stored (rounded) dz
        bs1 += dz;
        unsigned xraw;
        if constexpr (KEEP_XR) {
          xraw = xr[j];
        } else {
          xraw = rd(sxh, j + 1);
          if constexpr (ASMRD) ring_fence1(xraw);
        }
        bs2 = vfma(dz, (R::unpack(xraw) - mu) * is, bs2);
      }
      if constexpr (RES) s += R::unpack(pres[j]);
      if (skip_row && !a.skip_pre) s += R::unpack(pskp[j]);
      if constexpr (RES) {
        if constexpr (bnres) {
          const bool valid = cok && x0 + j < a.W;
          const V dz = valid ? R::unpack(R::pack(s)) : V(0.f);   // the stored (rounded) dX
          bs1 += dz;
          bs2 = vfma(dz, (R::unpack(pyb[j]) - mu) * is, bs2);
        }
      }
      *reinterpret_cast<unsigned*>(stg + (sg * RS + j) * SLICE + cl * 4) = R::pack(s);
    }
    store_row<T>(dX, h, a.W, a.C, rl_st, stg, lane);
  };
  // prologue: X rows r0 .. r0+BD-1, dY rows r0 .. r0+BD, dRes rows r0 .. r0+BD-1; dY row r0-1
  // (zero above the frame) first, into the register window (rolling form) or its ring slot
  V gup[ROLL ? RS + 2 : 1];
  if (r0 > 0) {
    stage_row<T>(G, r0 - 1, a.H, a.W, a.C, rl_ld, sgs(r0 - 1), lane);
    if constexpr (ROLL) {
      vmwait<0>();
      cvtg(sgs(r0 - 1), gup);
      __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0): the row is in registers before its slot is refilled
    }
  } else if constexpr (ROLL) {
#pragma unroll
    for (int k = 0; k < RS + 2; ++k) gup[k] = V(0.f);
  }
#pragma unroll
  for (int r = 0; r <= BD; ++r) {
    if (r < BD) stage_row<T>(X, r0 + r, hx, a.W, a.C, rl_ld, sx(r0 + r), lane);
    stage_row<T>(G, r0 + r, hg, a.W, a.C, rl_ld, sgs(r0 + r), lane);
    if constexpr (RES)
      if (r < BD) stage_row<T>(dRes, r0 + r, hx, a.W, a.C, rl_ld, sr(r0 + r), lane);
  }
  vmwait<0>();
  if constexpr (ROLL) {
    V g1[RS + 2], g2[RS + 2];
    cvtg(sgs(r0), g1);
    for (int h = r0; h < r1; h += 3) {
      step(h, gup, g1, g2);
      if (h + 1 < r1) step(h + 1, g1, g2, gup);
      if (h + 2 < r1) step(h + 2, g2, gup, g1);
    }
  } else {
    V gx[RS + 2];   // (unused by the streaming step)
    for (int h = r0; h < r1; ++h) step(h, gx, gx, gx);
  }
  // reduce the 4 lane segments (lanes cl, cl+16, cl+32, cl+48) and write the partials
  float red[EPT][11];
#pragma unroll
  for (int e = 0; e < EPT; ++e) {
#pragma unroll
    for (int t = 0; t < 9; ++t) red[e][t] = R::get(dw[t], e);
    red[e][9] = R::get(bs1, e);
    red[e][10] = R::get(bs2, e);
#pragma unroll
    for (int q = 0; q < 11; ++q) {
      red[e][q] += __shfl_xor(red[e][q], 16, 64);
      red[e][q] += __shfl_xor(red[e][q], 32, 64);
    }
  }
  if (sg == 0 && cok) {
#pragma unroll
    for (int e = 0; e < EPT; ++e) {
#pragma unroll
      for (int t = 0; t < 9; ++t) a.dWpart[((long)mp.unit * a.C + c + e) * 9 + t] = red[e][t];
      if (bnsum) {
        a.bnpart[((long)mp.unit * 2 + 0) * a.C + c + e] = red[e][9];
        a.bnpart[((long)mp.unit * 2 + 1) * a.C + c + e] = red[e][10];
      }
    }
  }
}

// XCP_DW_BWD_ROLL=1: the rolling-window form for every variant (the round-2 kernel; A/B)
bool dw_bwd_roll_all() {
  static const bool v = [] {
    const char* e = getenv("XCP_DW_BWD_ROLL");
    return e && e[0] == '1';
  }();
  return v;
}
// Default for calls without a strided-skip input: the streaming form with one row of look-ahead
// (6 ring rows per wave, 39 KB per workgroup, 112-122 VGPRs: four waves per SIMD; with a residual
// 8 rows, 50 KB, three).  Against the BD = 2 forms at the step's shapes (tools/dw_ab.py,
// profiles/r03_dw_occ4_ab.txt): 137.0 -> 119.4 us at 19^2 x 736, 154.2 -> 144.0 with the residual,
// 426 -> 398 at 37^2, 113 -> 96 at 10^2 x 1536; outputs bitwise equal except the residual form's dX
// (bf16 rounding of the reordered window sum).  XCP_DW_BWD_OCC4=0 keeps the BD = 2 forms (A/B).
bool dw_bwd_occ4() {
  static const bool v = [] {
    const char* e = getenv("XCP_DW_BWD_OCC4");
    return !(e && e[0] == '0');
  }();
  return v;
}

// Row bands per frame: the row walk of a frame split into b bands of ceil(H / b) rows (one wave
// each; a band re-reads the dY rows just above and below it).  Default: 3 bands for frames of 64
// rows or more (147^2 x 128: 1,101 -> 1,041 us; 74^2 x 256: 560 -> 548), one below (at 19^2 two
// bands cost 119.5 -> 125 us: the extra halo rows outweigh the shorter tail; profiles/r04_dw_tn_ab.txt).
// XCP_DW_BWD_BANDS=<b> forces b for every frame of >= 2 b rows.  (Read per call, so a test can
// compare band counts in one process.)
int dw_bwd_bands(int H) {
  const char* e = getenv("XCP_DW_BWD_BANDS");
  int v = e ? atoi(e) : (H >= 64 ? 3 : 1);
  v = v >= 1 && v <= 8 ? v : 1;
  return H >= 2 * v ? v : 1;
}

// XCD-aware workgroup order for the backward walk (default; 19^2 x 736: 119.5 -> 117.8 us, with the
// residual 143.5 -> 137.8; the step +0.3 %, profiles/r04_dw_tn_ab.txt).  XCP_DW_BWD_XCD=0 turns it off
// (read per call).
int dw_bwd_xcd() {
  const char* e = getenv("XCP_DW_BWD_XCD");
  return e && e[0] == '0' ? 0 : 1;
}

// Ring reads: plain C++ reads by default.  Round 4 measured inline-asm reads faster below 32 rows
// (118.4 -> 111.0 us at 19^2 x 736, profiles/r04_dw_asm_ab.txt) because hipcc drained vmcnt(0) ahead
// of the first plain ring read of every step; with the rings and the staging in one LDS object (round
// 5) that drain is gone and the plain form (offsets folded into the reads, no per-window fences) is as
// fast or faster at every step shape (19^2: 103.6 / 102.6 us plain / asm, 10^2: 90.9 / 96.7;
// profiles/r05_dw_bwd_onelds_ab.txt).  XCP_DW_BWD_ASM=1 forces the asm form (read per call).
bool dw_bwd_asm_reads(int) {
  const char* e = getenv("XCP_DW_BWD_ASM");
  return e && e[0] == '1';
}

// XCP_DW_BWD_SKIP4=0: calls with a strided-skip gradient (the first unit of blocks 2, 3 and 12) keep the
// two-rows-of-look-ahead form instead of the one-row form with plain ring reads (A/B; read per call)
bool dw_bwd_skip4() {
  const char* e = getenv("XCP_DW_BWD_SKIP4");
  return !(e && e[0] == '0');
}

template <typename T, int ACT>
void launch_bwd_act(const DwBwdArgs& a, int blocks, hipStream_t st) {
  // every form reads the ring with plain C++ reads unless XCP_DW_BWD_ASM=1 (the inline-asm form, kept
  // for the bitwise A/B test_dw_bwd_ring_read_forms)
  const bool asmrd = dw_bwd_asm_reads(a.H);
#define DWB(...)                                                                                  \
  do {                                                                                            \
    if (asmrd) hipLaunchKernelGGL((dw_bwd_lds_kernel<__VA_ARGS__, true>), dim3(blocks), dim3(256), 0, st, a); \
    else hipLaunchKernelGGL((dw_bwd_lds_kernel<__VA_ARGS__, false>), dim3(blocks), dim3(256), 0, st, a);     \
  } while (0)
  if (a.dRes && dw_bwd_occ4() && !a.dSkip) {
    if (a.Yb) DWB(T, ACT, true, false, 1, 3, false, true);
    else DWB(T, ACT, true, false, 1, 3, false, false);
  } else if (a.dRes && a.Yb)
    DWB(T, ACT, true, true, 2, 2, true, true);
  else if (a.dRes) DWB(T, ACT, true, true, 2, 2, true, false);
  else if (dw_bwd_roll_all()) DWB(T, ACT, false, true, 2, 2, true, false);
  else if (dw_bwd_occ4() && a.dSkip && dw_bwd_skip4())
    DWB(T, ACT, false, false, 1, 3, true, false);
  else if (dw_bwd_occ4() && !a.dSkip)
    DWB(T, ACT, false, false, 1, 4, false, false);
  else DWB(T, ACT, false, false, 2, 3, true, false);
#undef DWB
}

template <typename T>
int launch_bwd_lds(int act, const DwBwdArgs& a, hipStream_t st) {
  const long waves = (long)a.N * ((a.W + RCOLS - 1) / RCOLS) * a.nbands * a.ngroups;
  const int blocks = (int)((waves + 3) / 4);
  if (act == ACT_NONE) launch_bwd_act<T, ACT_NONE>(a, blocks, st);
  else if (act == ACT_RELU) launch_bwd_act<T, ACT_RELU>(a, blocks, st);
  else launch_bwd_act<T, ACT_BNRELU>(a, blocks, st);
  return (int)hipGetLastError();
}

}  // namespace

int xcp_internal_dw_fwd_small(int act, const void* X, void* Y, const float* Wt, const float* scale, const float* shift,
                              int N, int H, int W, int C, hipStream_t st);   // dwframe.hip

extern "C" {

int xcp_dw_fwd(int dtype, int act, const void* X, void* Y, const float* Wt, const float* scale, const float* shift, int N,
               int H, int W, int C, hipStream_t stream) {
  if (C % 8) return XCP_EINVAL;
  if (N <= 0 || H <= 0 || W <= 0) return XCP_OK;
  if (dtype == XCP_BF16 && W <= 8) {   // tiny frames (the 64^2 audio family's exit flow): dwframe.hip
    const int rc = xcp_internal_dw_fwd_small(act, X, Y, Wt, scale, shift, N, H, W, C, stream);
    if (rc != XCP_EUNSUPPORTED) return rc;
  }
  if (dtype != XCP_BF16 && dtype != XCP_F32) return XCP_EUNSUPPORTED;
  // the staging and the stores address one frame by 32-bit byte offsets
  if ((long)H * W * C * (dtype == XCP_BF16 ? 2 : 4) >= 0x7fffffffL) return XCP_EUNSUPPORTED;
  if (fwd_slice_bytes(C, dtype == XCP_BF16 ? 2 : 4, H, W) == 128) {
    DwArgs a{X, Y, Wt, scale, shift, N, H, W, C, ngroups_for(C, dtype, 128), tile_geo(H, W, FWD_MAXPX128)};
    if (dtype == XCP_BF16) return launch_fwd<bf16, FWD_MAXPX128, 128>(act, a, stream);
    return launch_fwd<float, FWD_MAXPX128, 128>(act, a, stream);
  }
  DwArgs a{X, Y, Wt, scale, shift, N, H, W, C, ngroups_for(C, dtype), tile_geo(H, W, FWD_MAXPX)};
  if (dtype == XCP_BF16 && dw_fwd_w2()) {
    const int sg = dw_fwd_w2();
    a.g = tile_geo(H, W, FWD_MAXPX, sg);
    const int blocks = a.N * a.g.nth * a.g.ntw * a.ngroups;
#define XCP_W2(SGV)                                                                                                  \
    if (act == ACT_NONE) hipLaunchKernelGGL((dw_fwd_w2_kernel<ACT_NONE, FWD_MAXPX, SGV>), dim3(blocks), dim3(256), 0, stream, a); \
    else if (act == ACT_RELU) hipLaunchKernelGGL((dw_fwd_w2_kernel<ACT_RELU, FWD_MAXPX, SGV>), dim3(blocks), dim3(256), 0, stream, a); \
    else hipLaunchKernelGGL((dw_fwd_w2_kernel<ACT_BNRELU, FWD_MAXPX, SGV>), dim3(blocks), dim3(256), 0, stream, a);
    if (sg == 4) { XCP_W2(4) } else { XCP_W2(5) }
#undef XCP_W2
    return (int)hipGetLastError();
  }
  if (dtype == XCP_BF16) return launch_fwd<bf16, FWD_MAXPX, 64>(act, a, stream);
  return launch_fwd<float, FWD_MAXPX, 64>(act, a, stream);
}

// number of partial rows (frame x 20-column group x row band) of the backward's slabs
int xcp_dw_bwd_chunks(int N, int H, int W, int C) {
  (void)C;
  return N * ((W + RCOLS - 1) / RCOLS) * dw_bwd_bands(H);
}

static int dw_bwd_impl(int dtype, int act, const void* dY, const void* X, const float* Wt, const float* scale,
                       const float* shift, const void* dRes, const void* dSkip, int sOH, int sOW, int sS, int skip_pre,
                       void* dX, float* dWpart, float* bnpart, const float* bmean, const float* binvstd, const void* Yb,
                       int N, int H, int W, int C, hipStream_t stream) {
  if (C % 8) return XCP_EINVAL;
  if (N <= 0 || H <= 0 || W <= 0) return XCP_OK;
  // the row walk stages a frame by 32-bit byte offsets
  if ((long)H * W * C * (dtype == XCP_BF16 ? 2 : 4) >= 0x7fffffffL) return XCP_EUNSUPPORTED;
  if (Yb) {   // sums over the final dX: needs the residual input, no skip input, and the BN's statistics
    if (!dRes || dSkip || !bnpart || !bmean || !binvstd) return XCP_EINVAL;
  } else if (bnpart && (act != ACT_BNRELU || !bmean || !binvstd)) {
    return XCP_EINVAL;
  }
  DwBwdArgs a{};
  a.dY = dY; a.X = X; a.Wt = Wt; a.scale = scale; a.shift = shift; a.dRes = dRes; a.dSkip = dSkip;
  a.sOH = sOH; a.sOW = sOW; a.sS = sS > 0 ? sS : 1; a.skip_pre = skip_pre != 0; a.dX = dX; a.dWpart = dWpart;
  a.bnpart = bnpart; a.bmean = bmean; a.binvstd = binvstd; a.Yb = Yb;
  a.N = N; a.H = H; a.W = W; a.C = C;
  a.ngroups = ngroups_for(C, dtype);
  a.nbands = dw_bwd_bands(H);
  a.xcd = dw_bwd_xcd();
  a.bandH = (H + a.nbands - 1) / a.nbands;
  if (dtype == XCP_BF16) return launch_bwd_lds<bf16>(act, a, stream);
  if (dtype == XCP_F32) return launch_bwd_lds<float>(act, a, stream);
  return XCP_EUNSUPPORTED;
}

int xcp_dw_bwd(int dtype, int act, const void* dY, const void* X, const float* Wt, const float* scale, const float* shift,
               const void* dRes, const void* dSkip, int sOH, int sOW, int sS, int skip_pre, void* dX, float* dWpart,
               float* bnpart, const float* bmean, const float* binvstd, int N, int H, int W, int C, hipStream_t stream) {
  return dw_bwd_impl(dtype, act, dY, X, Wt, scale, shift, dRes, dSkip, sOH, sOW, sS, skip_pre, dX, dWpart, bnpart, bmean,
                     binvstd, nullptr, N, H, W, C, stream);
}

int xcp_dw_bwd_resbn(int dtype, int act, const void* dY, const void* X, const float* Wt, const float* scale,
                     const float* shift, const void* dRes, void* dX, float* dWpart, float* bnpart, const float* bmean,
                     const float* binvstd, const void* Yb, int N, int H, int W, int C, hipStream_t stream) {
  return dw_bwd_impl(dtype, act, dY, X, Wt, scale, shift, dRes, nullptr, 0, 0, 1, 0, dX, dWpart, bnpart, bmean, binvstd, Yb,
                     N, H, W, C, stream);
}

}  // extern "C"
