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
XCP_DEV unsigned pack(const float* v, bf16*) {
  bf16x4 q;  // hardware RNE conversion (v_cvt_pk_bf16_f32)
  q[0] = (bf16)v[0];
  q[1] = (bf16)v[1];
  const u16x4 r = __builtin_bit_cast(u16x4, q);
  return (unsigned)r[0] | ((unsigned)r[1] << 16);
}
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
  uint4 v[MAXIT];
  bool ok[MAXIT];
#pragma unroll
  for (int k = 0; k < MAXIT; ++k) {
    const int i = threadIdx.x + 256 * k;
    const int p = i / CPP, q = i - p * CPP;
    const int hy = p / g.WP, hx = p - hy * g.WP;
    const int h = th0 - 1 + hy, w = tw0 - 1 + hx;
    const int c = c0 + q * EPC;
    ok[k] = i < total && h >= 0 && h < H && w >= 0 && w < W && c < C;
    const T* ptr = ok[k] ? src + (nbase + (long)h * W + w) * C + c : src;
    v[k] = *reinterpret_cast<const uint4*>(ptr);
  }
#pragma unroll
  for (int k = 0; k < MAXIT; ++k) {
    const int i = threadIdx.x + 256 * k;
    if (i >= total) break;
    const int p = i / CPP, q = i - p * CPP;
    uint4 u = ok[k] ? v[k] : make_uint4(0, 0, 0, 0);
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
  T* Y = reinterpret_cast<T*>(a.Y);
  const int items = g.TH * g.nseg;
  const char* lbase = sA + cl * 4;
  for (int it = wk; it < items; it += NWK) {
    const int r = it / g.nseg, sg = it - r * g.nseg;
    const int oh = th0 + r;
    const int x0 = sg * SEGL;
    if (oh >= a.H) continue;
    const char* base = lbase + (r * g.WP + x0) * FS;
    float win[3][SEGL + 2][EPT];
#pragma unroll
    for (int ky = 0; ky < 3; ++ky)
#pragma unroll
      for (int k = 0; k < SEGL + 2; ++k)
        unpack(*reinterpret_cast<const unsigned*>(base + (ky * g.WP + k) * FS), win[ky][k], (T*)nullptr);
    T* yrow = Y + (nbase + (long)oh * a.W + tw0) * a.C + c;
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
      const int x = x0 + j;
      if (x < g.TW && tw0 + x < a.W) *reinterpret_cast<unsigned*>(yrow + (long)x * a.C) = pack(o, (T*)nullptr);
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
  bf16* Y = reinterpret_cast<bf16*>(a.Y);
  const int items = g.TH * g.nseg;
  const char* lbase = sA + cl * 8;
  for (int it = wk; it < items; it += NWK) {
    const int r = it / g.nseg, sg = it - r * g.nseg;
    const int oh = th0 + r;
    const int x0 = sg * SG;
    if (oh >= a.H) continue;
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
    bf16* yrow = Y + (nbase + (long)oh * a.W + tw0) * a.C + c;
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
      const int x = x0 + j;
      if (x < g.TW && tw0 + x < a.W)
        *reinterpret_cast<uint2*>(yrow + (long)x * a.C) = make_uint2(pack(o, (bf16*)nullptr), pack(o + 2, (bf16*)nullptr));
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
// Pipelined forward (dw_fwd_pipe_kernel): the tile of dw_fwd_w2_kernel, but persistent
// workgroups (two per CU, 64 KB of LDS each) that stream their tiles through a two-slot LDS ring
// by LDS-DMA, so a tile's loads are in flight while the previous tile computes and stores.  The
// one-tile-per-workgroup kernel has loads in flight only during its staging phase (~1/3 of a
// workgroup's life: ~16 GB/s per CU moved at 19^2 x 736, 0.42 of HBM); here every workgroup keeps
// the next tile's ~23 KB in flight throughout.
//   * The DMA lands raw bytes (out-of-frame halo pixels and channels past C read as zeros through
//     the buffer resource's out-of-range offset).  The producer's BN + ReLU is then applied in
//     place by one LDS pass over the tile's in-frame chunks (ACT_RELU needs no pass where the halo
//     is zero: relu(0) = 0, but applies max(., 0) in the same pass), so the register window, the
//     fma chain and the stored values are exactly those of dw_fwd_w2_kernel.
//   * Every thread issues the same number of DMA instructions (nd per tile) and of output stores
//     (ns per tile, masked ones as out-of-range buffer stores), so counted vmcnt waits retire a
//     tile's DMA without waiting for the previous tile's stores.
//   * Raw s_barrier / lgkmcnt only (no __syncthreads, whose fence would drain vmcnt).
constexpr unsigned DBUF_OOB = 0x80000000u;
constexpr long DBUF_LIMIT = 0x7fffffffL;
constexpr int DBUF_RECORDS = 0x7fffffff;
constexpr int DBUF_DWORD3 = 0x00020000;
constexpr int PIPE_MAXPX = 512;
constexpr int DW_PIPE_PX = PIPE_MAXPX * SLICE;        // 32 KB of pixel slices per ring slot
constexpr int DW_PIPE_SLOT = DW_PIPE_PX + 4096;       // + the tile's parameters: scale @0, shift @1 KB, taps (9 x 128 B) @2 KB

XCP_DEV void dvm_wait(int n) {   // s_waitcnt vmcnt(n), n clamped to [0, 63]
  switch (n < 0 ? 0 : n > 63 ? 63 : n) {
#define XCP_DVMW(k) case k: asm volatile("s_waitcnt vmcnt(" #k ")" ::: "memory"); break;
    XCP_DVMW(0) XCP_DVMW(1) XCP_DVMW(2) XCP_DVMW(3) XCP_DVMW(4) XCP_DVMW(5) XCP_DVMW(6) XCP_DVMW(7)
    XCP_DVMW(8) XCP_DVMW(9) XCP_DVMW(10) XCP_DVMW(11) XCP_DVMW(12) XCP_DVMW(13) XCP_DVMW(14) XCP_DVMW(15)
    XCP_DVMW(16) XCP_DVMW(17) XCP_DVMW(18) XCP_DVMW(19) XCP_DVMW(20) XCP_DVMW(21) XCP_DVMW(22) XCP_DVMW(23)
    XCP_DVMW(24) XCP_DVMW(25) XCP_DVMW(26) XCP_DVMW(27) XCP_DVMW(28) XCP_DVMW(29) XCP_DVMW(30) XCP_DVMW(31)
    XCP_DVMW(32) XCP_DVMW(33) XCP_DVMW(34) XCP_DVMW(35) XCP_DVMW(36) XCP_DVMW(37) XCP_DVMW(38) XCP_DVMW(39)
    XCP_DVMW(40) XCP_DVMW(41) XCP_DVMW(42) XCP_DVMW(43) XCP_DVMW(44) XCP_DVMW(45) XCP_DVMW(46) XCP_DVMW(47)
    XCP_DVMW(48) XCP_DVMW(49) XCP_DVMW(50) XCP_DVMW(51) XCP_DVMW(52) XCP_DVMW(53) XCP_DVMW(54) XCP_DVMW(55)
    XCP_DVMW(56) XCP_DVMW(57) XCP_DVMW(58) XCP_DVMW(59) XCP_DVMW(60) XCP_DVMW(61) XCP_DVMW(62) XCP_DVMW(63)
#undef XCP_DVMW
  }
}

typedef int di32x2 __attribute__((ext_vector_type(2)));

// LDS accesses of the pipelined kernel by inline asm, each block carrying its own lgkmcnt wait:
// hipcc puts an s_waitcnt vmcnt(0) before any compiler-visible LDS access that may alias an LDS-DMA
// destination, which would retire the next tile's DMA (the ring) at every read.  A load and the wait
// for it sit in ONE asm statement, so no use or copy of the result can be scheduled between them.
typedef unsigned du32x4 __attribute__((ext_vector_type(4)));
typedef unsigned du32x2 __attribute__((ext_vector_type(2)));
XCP_DEV unsigned dlds(const void* p) { return (unsigned)(size_t)(const __attribute__((address_space(3))) char*)(p); }
XCP_DEV void lds_ld4x128(const char* p0, const char* p1, const char* p2, const char* p3, du32x4& a, du32x4& b, du32x4& c,
                         du32x4& d) {
  asm volatile(
      "ds_read_b128 %0, %4\n\t"
      "ds_read_b128 %1, %5\n\t"
      "ds_read_b128 %2, %6\n\t"
      "ds_read_b128 %3, %7\n\t"
      "s_waitcnt lgkmcnt(0)"
      : "=&v"(a), "=&v"(b), "=&v"(c), "=&v"(d)
      : "v"(dlds(p0)), "v"(dlds(p1)), "v"(dlds(p2)), "v"(dlds(p3))
      : "memory");
}
XCP_DEV void lds_st128(char* p, const du32x4& v) {
  asm volatile("ds_write_b128 %0, %1" ::"v"(dlds(p)), "v"(v) : "memory");
}
XCP_DEV void lds_wait() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }
// the 3 x 7 window of a 5-pixel segment: rows r0, r1, r2 (byte addresses), pixels k * 64 B apart
XCP_DEV void lds_win7(const char* r0, const char* r1, const char* r2, du32x2 (&v)[3][7]) {
  asm volatile(
      "ds_read_b64 %0, %21\n\t"
      "ds_read_b64 %1, %21 offset:64\n\t"
      "ds_read_b64 %2, %21 offset:128\n\t"
      "ds_read_b64 %3, %21 offset:192\n\t"
      "ds_read_b64 %4, %21 offset:256\n\t"
      "ds_read_b64 %5, %21 offset:320\n\t"
      "ds_read_b64 %6, %21 offset:384\n\t"
      "ds_read_b64 %7, %22\n\t"
      "ds_read_b64 %8, %22 offset:64\n\t"
      "ds_read_b64 %9, %22 offset:128\n\t"
      "ds_read_b64 %10, %22 offset:192\n\t"
      "ds_read_b64 %11, %22 offset:256\n\t"
      "ds_read_b64 %12, %22 offset:320\n\t"
      "ds_read_b64 %13, %22 offset:384\n\t"
      "ds_read_b64 %14, %23\n\t"
      "ds_read_b64 %15, %23 offset:64\n\t"
      "ds_read_b64 %16, %23 offset:128\n\t"
      "ds_read_b64 %17, %23 offset:192\n\t"
      "ds_read_b64 %18, %23 offset:256\n\t"
      "ds_read_b64 %19, %23 offset:320\n\t"
      "ds_read_b64 %20, %23 offset:384\n\t"
      "s_waitcnt lgkmcnt(0)"
      : "=&v"(v[0][0]), "=&v"(v[0][1]), "=&v"(v[0][2]), "=&v"(v[0][3]), "=&v"(v[0][4]), "=&v"(v[0][5]), "=&v"(v[0][6]),
        "=&v"(v[1][0]), "=&v"(v[1][1]), "=&v"(v[1][2]), "=&v"(v[1][3]), "=&v"(v[1][4]), "=&v"(v[1][5]), "=&v"(v[1][6]),
        "=&v"(v[2][0]), "=&v"(v[2][1]), "=&v"(v[2][2]), "=&v"(v[2][3]), "=&v"(v[2][4]), "=&v"(v[2][5]), "=&v"(v[2][6])
      : "v"(dlds(r0)), "v"(dlds(r1)), "v"(dlds(r2))
      : "memory");
}
// the 3 x 6 window of a 4-pixel segment
XCP_DEV void lds_win6(const char* r0, const char* r1, const char* r2, du32x2 (&v)[3][6]) {
  asm volatile(
      "ds_read_b64 %0, %18\n\t"
      "ds_read_b64 %1, %18 offset:64\n\t"
      "ds_read_b64 %2, %18 offset:128\n\t"
      "ds_read_b64 %3, %18 offset:192\n\t"
      "ds_read_b64 %4, %18 offset:256\n\t"
      "ds_read_b64 %5, %18 offset:320\n\t"
      "ds_read_b64 %6, %19\n\t"
      "ds_read_b64 %7, %19 offset:64\n\t"
      "ds_read_b64 %8, %19 offset:128\n\t"
      "ds_read_b64 %9, %19 offset:192\n\t"
      "ds_read_b64 %10, %19 offset:256\n\t"
      "ds_read_b64 %11, %19 offset:320\n\t"
      "ds_read_b64 %12, %20\n\t"
      "ds_read_b64 %13, %20 offset:64\n\t"
      "ds_read_b64 %14, %20 offset:128\n\t"
      "ds_read_b64 %15, %20 offset:192\n\t"
      "ds_read_b64 %16, %20 offset:256\n\t"
      "ds_read_b64 %17, %20 offset:320\n\t"
      "s_waitcnt lgkmcnt(0)"
      : "=&v"(v[0][0]), "=&v"(v[0][1]), "=&v"(v[0][2]), "=&v"(v[0][3]), "=&v"(v[0][4]), "=&v"(v[0][5]),
        "=&v"(v[1][0]), "=&v"(v[1][1]), "=&v"(v[1][2]), "=&v"(v[1][3]), "=&v"(v[1][4]), "=&v"(v[1][5]),
        "=&v"(v[2][0]), "=&v"(v[2][1]), "=&v"(v[2][2]), "=&v"(v[2][3]), "=&v"(v[2][4]), "=&v"(v[2][5])
      : "v"(dlds(r0)), "v"(dlds(r1)), "v"(dlds(r2))
      : "memory");
}

struct DwPipeArgs {
  DwArgs a;
  int ntiles;   // N * nth * ntw * ngroups
  int nd;       // DMA instructions per wave per tile: ceil(HP * WP * 4 / 256)
  int nit;      // row items per worker per tile: ceil(TH * nseg / 32)
};

template <int ACT, int SG, int NWV, int NSLOT>
__global__ __launch_bounds__(NWV * 64) void dw_fwd_pipe_kernel(DwPipeArgs pa) {
  constexpr int NT = NWV * 64, FS = SLICE, LANES = FS / 8, NWK = NT / LANES, CPL = 4;
  __shared__ __attribute__((aligned(16))) char ring[NSLOT * DW_PIPE_SLOT];
  // every field in a local scalar: the lambdas below take them by reference, and a reference to the
  // kernel-argument struct itself put it in scratch (private memory), with a vmcnt(0) at each use
  const int H = pa.a.H, W = pa.a.W, C = pa.a.C, ngroups = pa.a.ngroups;
  const int TH = pa.a.g.TH, TW = pa.a.g.TW, HP = pa.a.g.HP, WP = pa.a.g.WP, ntw = pa.a.g.ntw, nseg = pa.a.g.nseg;
  const int ntiles = pa.ntiles, ndp = pa.nd, nit = pa.nit;
  const void* Xp = pa.a.X;
  void* Yp = pa.a.Y;
  const float *Wtp = pa.a.Wt, *scp = pa.a.scale, *shp = pa.a.shift;
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int cl = tid % LANES, wk = tid / LANES;
  const int nwg = gridDim.x;
  const int ntl = pa.a.g.nth * ntw;
  const int total = HP * WP * 4;   // 16-B chunks of a staged tile
  const __amdgpu_buffer_rsrc_t rX = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(Xp), (short)0, DBUF_RECORDS,
                                                                       DBUF_DWORD3);
  const __amdgpu_buffer_rsrc_t rY = __builtin_amdgcn_make_buffer_rsrc(Yp, (short)0, DBUF_RECORDS, DBUF_DWORD3);
  // tile id -> (channel slice, frame, spatial tile), as block_coords with the logical id
  auto coords = [&](int id, int& grp, int& n, int& th0, int& tw0) {
    grp = id % ngroups;
    const int sp = id / ngroups;
    const int tile = sp % ntl;
    n = sp / ntl;
    th0 = (tile / ntw) * TH;
    tw0 = (tile % ntw) * TW;
  };
  const __amdgpu_buffer_rsrc_t rP = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(Wtp), (short)0, DBUF_RECORDS,
                                                                       DBUF_DWORD3);
  const __amdgpu_buffer_rsrc_t rS = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(ACT == ACT_BNRELU ? scp : Wtp), (short)0, DBUF_RECORDS, DBUF_DWORD3);
  const __amdgpu_buffer_rsrc_t rT = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(ACT == ACT_BNRELU ? shp : Wtp), (short)0, DBUF_RECORDS, DBUF_DWORD3);
  // the DMA of tile `id` into ring slot `dst`: nd pixel pieces per wave (wave w's pieces j = w*nd + k),
  // and by wave 0 two more pieces with the tile's parameters -- scale / shift of its 32 channels
  // (chunks 0-15) and its 9 x 32 taps (chunks 16-87) -- so that nothing a tile reads is a register
  // load younger than the DMA in flight (a vmcnt wait for one would drain the ring)
  auto issue = [&](int id, char* dst) {
    int grp, n, th0, tw0;
    coords(id, grp, n, th0, tw0);
    const int c0 = grp * 32;
    const long nbase = (long)n * H * W;
    if (w == 0) {   // (one buffer resource per instruction: a per-lane resource select is a waterfall loop)
      char* pd = dst + DW_PIPE_PX;
      if constexpr (ACT == ACT_BNRELU) {
        const unsigned o = lane < 8 && c0 + lane * 4 < C ? (unsigned)((c0 + lane * 4) * 4) : DBUF_OOB;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rS, (__attribute__((address_space(3))) void*)pd, 16, o, 0, 0, 0);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rT, (__attribute__((address_space(3))) void*)(pd + 1024), 16, o, 0, 0, 0);
      }
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        const int c = k * 64 + lane, row = c >> 3, ch = c0 + (c & 7) * 4;
        const unsigned o = c < 72 && ch < C ? (unsigned)(((long)row * C + ch) * 4) : DBUF_OOB;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rP, (__attribute__((address_space(3))) void*)(pd + 2048 + k * 1024), 16, o,
                                                 0, 0, 0);
      }
    }
    for (int k = 0; k < ndp; ++k) {
      const int j = w * ndp + k;
      const int c = j * 64 + lane;
      const int p = c >> 2, q = c & 3;
      const int hy = p / WP, hx = p - hy * WP;
      const int h = th0 - 1 + hy, x = tw0 - 1 + hx;
      const int ch = c0 + q * 8;
      const bool ok = c < total && h >= 0 && h < H && x >= 0 && x < W && ch < C;
      const unsigned o = ok ? (unsigned)(((nbase + (long)h * W + x) * C + ch) * 2) : DBUF_OOB;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rX, (__attribute__((address_space(3))) void*)(dst + j * 1024), 16, o, 0,
                                               0, 0);
    }
  };
  // one tile: (BN +) ReLU in place, then the 3 x (SG+2) register windows and nit * SG output stores
  auto work = [&](int id, char* sA) {
    int grp, n, th0, tw0;
    coords(id, grp, n, th0, tw0);
    const int c0 = grp * 32;
    const long nbase = (long)n * H * W;
    const float* prm = reinterpret_cast<const float*>(sA + DW_PIPE_PX);   // scale[32] @0, shift[32] @256, taps[9][32] @512
    if constexpr (ACT != ACT_NONE) {
      // this thread's chunks are tid + NT k: always channel chunk q = tid & 3
      const int q = tid & 3;
      float sc[8], sh[8];
      if constexpr (ACT == ACT_BNRELU) {
        du32x4 r[4];
        lds_ld4x128(reinterpret_cast<const char*>(prm + q * 8), reinterpret_cast<const char*>(prm + q * 8 + 4),
                    reinterpret_cast<const char*>(prm + 256 + q * 8), reinterpret_cast<const char*>(prm + 256 + q * 8 + 4),
                    r[0], r[1], r[2], r[3]);
        VecIO<float, 4>::load(reinterpret_cast<const float*>(&r[0]), sc);
        VecIO<float, 4>::load(reinterpret_cast<const float*>(&r[1]), sc + 4);
        VecIO<float, 4>::load(reinterpret_cast<const float*>(&r[2]), sh);
        VecIO<float, 4>::load(reinterpret_cast<const float*>(&r[3]), sh + 4);
      }
      // four chunks per asm read block (out-of-tile chunks read chunk 0 and are not written back)
      for (int c4 = tid; c4 < total; c4 += 4 * NT) {
        du32x4 u[4];
        const int cs[4] = {c4, c4 + NT, c4 + 2 * NT, c4 + 3 * NT};
        lds_ld4x128(sA + (cs[0] < total ? cs[0] : 0) * 16, sA + (cs[1] < total ? cs[1] : 0) * 16,
                    sA + (cs[2] < total ? cs[2] : 0) * 16, sA + (cs[3] < total ? cs[3] : 0) * 16, u[0], u[1], u[2], u[3]);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int c = cs[r];
          const int p = c >> 2;
          const int hy = p / WP, hx = p - hy * WP;
          const int h = th0 - 1 + hy, x = tw0 - 1 + hx;
          // halo / padding chunks stay 0 (relu(bn(0)) need not be)
          if (c >= total || h < 0 || h >= H || x < 0 || x >= W || c0 + q * 8 >= C) continue;
          float f[8];
          VecIO<bf16, 8>::load(reinterpret_cast<const bf16*>(&u[r]), f);
          typedef float p2 __attribute__((ext_vector_type(2)));
#pragma unroll
          for (int e = 0; e < 8; e += 2) {
            p2 v = p2{f[e], f[e + 1]};
            if constexpr (ACT == ACT_BNRELU) v = __builtin_elementwise_fma(v, p2{sc[e], sc[e + 1]}, p2{sh[e], sh[e + 1]});
            v = __builtin_elementwise_max(v, p2(0.f));
            f[e] = v[0];
            f[e + 1] = v[1];
          }
          VecIO<bf16, 8>::store(reinterpret_cast<bf16*>(&u[r]), f);
          lds_st128(sA + c * 16, u[r]);
        }
      }
      lds_wait();
      __builtin_amdgcn_s_barrier();
    }
    const int c = c0 + cl * CPL;
    float wt[9][CPL];
    {
      du32x4 r[12];
      const char* wb = reinterpret_cast<const char*>(prm + 512 + cl * CPL);
      lds_ld4x128(wb, wb + 128, wb + 256, wb + 384, r[0], r[1], r[2], r[3]);
      lds_ld4x128(wb + 512, wb + 640, wb + 768, wb + 896, r[4], r[5], r[6], r[7]);
      lds_ld4x128(wb + 1024, wb + 1024, wb + 1024, wb + 1024, r[8], r[9], r[10], r[11]);
#pragma unroll
      for (int t = 0; t < 9; ++t) VecIO<float, CPL>::load(reinterpret_cast<const float*>(&r[t]), wt[t]);
    }
    const int items = TH * nseg;
    const char* lbase = sA + cl * 8;
    for (int s = 0; s < nit; ++s) {
      const int it = wk + s * NWK;
      const bool real = it < items;
      const int r = real ? it / nseg : 0, sg = real ? it - r * nseg : 0;
      const int oh = th0 + r;
      const int x0 = sg * SG;
      const char* base = lbase + (r * WP + x0) * FS;
      float win[3][SG + 2][CPL];
      du32x2 raw[3][SG + 2];
      if constexpr (SG == 5) lds_win7(base, base + WP * FS, base + 2 * WP * FS, raw);
      else lds_win6(base, base + WP * FS, base + 2 * WP * FS, raw);
#pragma unroll
      for (int ky = 0; ky < 3; ++ky)
#pragma unroll
        for (int k = 0; k < SG + 2; ++k) {
          unpack(raw[ky][k][0], win[ky][k], (bf16*)nullptr);
          unpack(raw[ky][k][1], win[ky][k] + 2, (bf16*)nullptr);
        }
      const long rowe = (nbase + (long)oh * W + tw0) * C + c;
#pragma unroll
      for (int j = 0; j < SG; ++j) {
        float o[CPL];
#pragma unroll
        for (int e = 0; e < CPL; ++e) {
          float sum = 0.f;
#pragma unroll
          for (int ky = 0; ky < 3; ++ky)
#pragma unroll
            for (int kx = 0; kx < 3; ++kx) sum = fmaf(win[ky][j + kx][e], wt[ky * 3 + kx][e], sum);
          o[e] = sum;
        }
        const int x = x0 + j;
        const bool ok = real && c < C && oh < H && x < TW && tw0 + x < W;
        const unsigned off = ok ? (unsigned)((rowe + (long)x * C) * 2) : DBUF_OOB;
        const uint2 v = make_uint2(pack(o, (bf16*)nullptr), pack(o + 2, (bf16*)nullptr));
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(di32x2, v), rY, (int)off, 0, 0);
      }
    }
    __builtin_amdgcn_s_barrier();   // every wave is done with this slot before the next DMA into it
  };
  const int ns = nit * SG;                    // stores per thread per tile
  const int nd = ndp + (w == 0 ? (ACT == ACT_BNRELU ? 4 : 2) : 0);   // DMA pieces per wave per tile
  const int t0 = xcd_remap(blockIdx.x, nwg);
  if (t0 >= ntiles) return;
  const int mine = (ntiles - 1 - t0) / nwg + 1;   // tiles of this workgroup: t0 + k nwg, k < mine
  // prologue: the first NSLOT - 1 tiles in flight
#pragma unroll
  for (int k = 0; k < NSLOT - 1; ++k)
    if (k < mine) issue(t0 + k * nwg, ring + k * DW_PIPE_SLOT);
  for (int k = 0; k < mine; ++k) {
    const int kn = k + NSLOT - 1;   // into the slot tile k - 1 has just left (its readers passed a barrier)
    if (kn < mine) issue(t0 + kn * nwg, ring + (kn % NSLOT) * DW_PIPE_SLOT);
    // tile k's DMA landed: younger are the stores of tiles k-NSLOT+1 .. k-1 and the DMA of tiles
    // k+1 .. min(k+NSLOT-1, mine-1) (vmcnt retires in issue order)
    const int younger = ns * min(NSLOT - 1, k) + nd * (min(kn, mine - 1) - k);
    dvm_wait(younger);
    __builtin_amdgcn_s_barrier();   // ... every wave's pieces of it
    work(t0 + k * nwg, ring + (k % NSLOT) * DW_PIPE_SLOT);
  }
}

// XCP_DW_FWD_PIPE=0: the one-tile-per-workgroup kernel; m = 1..4 the pipelined form
//   1: 4 waves, 2 slots, 2 workgroups per CU     2: 8 waves, 4 slots, 1 per CU
//   3: 8 waves, 2 slots, 2 per CU                4: 4 waves, 4 slots, 1 per CU
int dw_fwd_pipe() {   // (read per call: the bitwise test compares both kernels in one process)
  const char* e = getenv("XCP_DW_FWD_PIPE");
  const int m = e ? atoi(e) : 0;
  return m >= 0 && m <= 4 ? m : 0;
}
int dw_gpu_cus() {
  static const int cus = [] {
    int d = 0, n = 0;
    if (hipGetDevice(&d) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, d) != hipSuccess)
      n = 0;
    return n > 0 ? n : 256;
  }();
  return cus;
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
  BnFin fin;              // fin.acc: the BN partial sums folded into that BN's backward finalize (common.h)
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
  static XCP_DEV unsigned pack(V v) {
    bf16x4 q;
    q[0] = (bf16)v[0];
    q[1] = (bf16)v[1];
    const u16x4 r = __builtin_bit_cast(u16x4, q);
    return (unsigned)r[0] | ((unsigned)r[1] << 16);
  }
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
template <typename T>
XCP_DEV void stage_row(const T* frame, int h, int H, int W, int C, const RowLanes& rl, char* dst, int lane) {
  const T* row = frame + (long)h * W * C;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const void* src = (h < H && rl.off[i] >= 0) ? (const void*)(row + rl.off[i]) : (const void*)g_dzero;
    if (i == 0 || lane < 24)
      __builtin_amdgcn_global_load_lds((const void __attribute__((address_space(1)))*)src,
                                       (void __attribute__((address_space(3)))*)(dst + i * 1024), 16, 0, 0);
  }
}

// Write the staged output row (20 pixels x 64 B in `stg`) to row h: two 16-B stores
// per lane-slot; lanes without a valid pixel write the sink.
template <typename T>
XCP_DEV void store_row(T* frame, int h, int W, int C, const RowLanes& rl, const char* stg, int lane) {
  T* row = frame + (long)h * W * C;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int ch = i * 64 + lane;
    const uint4 v = *reinterpret_cast<const uint4*>(stg + min(ch, 4 * RCOLS - 1) * 16);
    uint4* dstp = rl.off[i] >= 0 ? reinterpret_cast<uint4*>(row + rl.off[i]) : g_dsink + lane;
    *dstp = v;
  }
}

// LDS reads of the DMA ring by inline asm: a plain C++ read of LDS that an LDS-DMA may write makes
// hipcc drain every outstanding vector-memory operation first (s_waitcnt vmcnt(0)) -- here right
// after a step had issued the look-ahead rows, so every step waited for the rows it had just asked
// for and the look-ahead never overlapped anything.  The counted vmwait at the top of a step is what
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
          bool BNRES = false, bool ASMRD = true>
__global__ __launch_bounds__(256, MINW) void dw_bwd_lds_kernel(DwBwdArgs a) {
  typedef RV<T> R;
  typedef typename R::V V;
  constexpr int EPT = R::EPT, CPG = 16 * EPT;
  constexpr int BD = BDV;                                // rows of look-ahead per staged tensor
  constexpr int NS = BD + 1;                             // X / dRes ring slots
  constexpr int NSG = ROLL ? NS : BD + 3;                // dY ring slots
  __shared__ __attribute__((aligned(16))) char sm[4][(NS + NSG + (RES ? NS : 0)) * LROW];
  __shared__ __attribute__((aligned(16))) char so[4][RCOLS * SLICE];   // output staging (separate object)
  const int ncg = (a.W + RCOLS - 1) / RCOLS;
  const RowMap mp = row_map(a.N, ncg, a.ngroups, a.nbands, a.xcd != 0);
  __shared__ int fin_last;
  if (!mp.live) {   // (a folded finalize: every wave of the workgroup takes part in its arrival)
    if (a.fin.acc && fin_arrive(a.fin, &fin_last)) fin_finalize(a.fin, threadIdx.x, 256);
    return;
  }
  // this wave's rows [r0, r1); it reads X rows r0 .. r1-1 and dY rows r0-1 .. r1 (rows past
  // those are staged from the zero line: never read)
  const int r0 = mp.band * a.bandH, r1 = min(a.H, r0 + a.bandH);
  const int hx = r1, hg = min(a.H, r1 + 1);
  const int lane = threadIdx.x & 63, cl = lane & 15, sg = lane >> 4;
  char* ring = sm[threadIdx.x >> 6];
  char* rx = ring;                  // X rows, slot r % NS
  char* rg = ring + NS * LROW;      // dY rows, slot r % NSG
  char* rres = rg + NSG * LROW;     // dRes rows (RES), slot r % NS
  char* stg = so[threadIdx.x >> 6];
  const int c0 = mp.grp * CPG;
  const int c = c0 + cl * EPT;
  const bool cok = c < a.C;
  const int cc = cok ? c : a.C - EPT;
  const int x0w = mp.cg * RCOLS, x0 = x0w + sg * RS;
  const RowLanes rl_ld = row_lanes_load<T>(a.W, a.C, x0w, c0, lane);
  const RowLanes rl_st = row_lanes_store<T>(a.W, a.C, x0w, c0, lane);
  const bool bnsum = a.bnpart != nullptr || a.fin.acc != nullptr;
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
  const T* X = reinterpret_cast<const T*>(a.X) + fbase;
  const T* G = reinterpret_cast<const T*>(a.dY) + fbase;
  const T* dRes = RES ? reinterpret_cast<const T*>(a.dRes) + fbase : nullptr;
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
      if (a.fin.acc) {
        fin_add(a.fin.acc + c + e, red[e][9]);
        fin_add(a.fin.acc + a.fin.CP + c + e, red[e][10]);
      } else if (bnsum) {
        a.bnpart[((long)mp.unit * 2 + 0) * a.C + c + e] = red[e][9];
        a.bnpart[((long)mp.unit * 2 + 1) * a.C + c + e] = red[e][10];
      }
    }
  }
  if (a.fin.acc && fin_arrive(a.fin, &fin_last)) fin_finalize(a.fin, threadIdx.x, 256);
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

// Ring reads by inline asm (no vmcnt(0) drain ahead of them) for frames below 32 rows, plain reads
// above: at the step's shapes the asm form measured 118.4 -> 111.0 us at 19^2 x 736 but 398 -> 408 at
// 37^2, 536 -> 544 at 74^2 and 1,034 -> 1,110 at 147^2 (tools/dw_ab.py, profiles/r04_dw_asm_ab.txt):
// with long walks the drain costs less than the per-read lgkmcnt(0) fences that replace it.
// XCP_DW_BWD_ASM=0 / 1 forces the plain / asm form for every frame (read per call).
bool dw_bwd_asm_reads(int H) {
  const char* e = getenv("XCP_DW_BWD_ASM");
  if (e && (e[0] == '0' || e[0] == '1')) return e[0] == '1';
  return H < 32;
}

template <typename T, int ACT>
void launch_bwd_act(const DwBwdArgs& a, int blocks, hipStream_t st) {
  if (a.dRes && dw_bwd_occ4() && !a.dSkip)
  {
    if (a.Yb) hipLaunchKernelGGL((dw_bwd_lds_kernel<T, ACT, true, false, 1, 3, false, true>), dim3(blocks), dim3(256), 0, st, a);
    else hipLaunchKernelGGL((dw_bwd_lds_kernel<T, ACT, true, false, 1, 3, false>), dim3(blocks), dim3(256), 0, st, a);
  } else if (a.dRes && a.Yb)
    hipLaunchKernelGGL((dw_bwd_lds_kernel<T, ACT, true, true, 2, 2, true, true>), dim3(blocks), dim3(256), 0, st, a);
  else if (a.dRes) hipLaunchKernelGGL((dw_bwd_lds_kernel<T, ACT, true, true>), dim3(blocks), dim3(256), 0, st, a);
  else if (dw_bwd_roll_all()) hipLaunchKernelGGL((dw_bwd_lds_kernel<T, ACT, false, true>), dim3(blocks), dim3(256), 0, st, a);
  else if (dw_bwd_occ4() && !a.dSkip) {
    if (dw_bwd_asm_reads(a.H))
      hipLaunchKernelGGL((dw_bwd_lds_kernel<T, ACT, false, false, 1, 4, false>), dim3(blocks), dim3(256), 0, st, a);
    else
      hipLaunchKernelGGL((dw_bwd_lds_kernel<T, ACT, false, false, 1, 4, false, false, false>), dim3(blocks), dim3(256), 0,
                         st, a);
  }
  else hipLaunchKernelGGL((dw_bwd_lds_kernel<T, ACT, false, false>), dim3(blocks), dim3(256), 0, st, a);
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
  if (fwd_slice_bytes(C, dtype == XCP_BF16 ? 2 : 4, H, W) == 128) {
    DwArgs a{X, Y, Wt, scale, shift, N, H, W, C, ngroups_for(C, dtype, 128), tile_geo(H, W, FWD_MAXPX128)};
    if (dtype == XCP_BF16) return launch_fwd<bf16, FWD_MAXPX128, 128>(act, a, stream);
    return launch_fwd<float, FWD_MAXPX128, 128>(act, a, stream);
  }
  DwArgs a{X, Y, Wt, scale, shift, N, H, W, C, ngroups_for(C, dtype), tile_geo(H, W, FWD_MAXPX)};
  if (dtype == XCP_BF16 && dw_fwd_w2()) {
    const int sg = dw_fwd_w2();
    a.g = tile_geo(H, W, FWD_MAXPX, sg);
    const long span = (long)N * H * W * C * 2;
    if (dw_fwd_pipe() && span <= DBUF_LIMIT && a.g.HP * a.g.WP <= PIPE_MAXPX) {
      DwPipeArgs pa{a, a.N * a.g.nth * a.g.ntw * a.ngroups, (a.g.HP * a.g.WP * 4 + 255) / 256,
                    (a.g.TH * a.g.nseg + 31) / 32};
      const int mode = dw_fwd_pipe();
      const int nwv = mode == 2 || mode == 3 ? 8 : 4, wgs = mode == 1 || mode == 3 ? 2 : 1;
      pa.nd = (a.g.HP * a.g.WP * 4 + 64 * nwv - 1) / (64 * nwv);
      pa.nit = (a.g.TH * a.g.nseg + nwv * 8 - 1) / (nwv * 8);
      const int grid = min(pa.ntiles, dw_gpu_cus() * wgs);
#define XCP_PIPE(SGV, NWV, NSL)                                                                                         \
      if (act == ACT_NONE) hipLaunchKernelGGL((dw_fwd_pipe_kernel<ACT_NONE, SGV, NWV, NSL>), dim3(grid), dim3(NWV * 64), 0, stream, pa); \
      else if (act == ACT_RELU) hipLaunchKernelGGL((dw_fwd_pipe_kernel<ACT_RELU, SGV, NWV, NSL>), dim3(grid), dim3(NWV * 64), 0, stream, pa); \
      else hipLaunchKernelGGL((dw_fwd_pipe_kernel<ACT_BNRELU, SGV, NWV, NSL>), dim3(grid), dim3(NWV * 64), 0, stream, pa);
      if (sg == 4) {
        XCP_PIPE(4, 4, 2)
      } else if (mode == 2) {
        XCP_PIPE(5, 8, 4)
      } else if (mode == 3) {
        XCP_PIPE(5, 8, 2)
      } else if (mode == 4) {
        XCP_PIPE(5, 4, 4)
      } else {
        XCP_PIPE(5, 4, 2)
      }
#undef XCP_PIPE
      return (int)hipGetLastError();
    }
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
                       int N, int H, int W, int C, hipStream_t stream, BnFin fin = BnFin{}) {
  if (C % 8) return XCP_EINVAL;
  if (N <= 0 || H <= 0 || W <= 0) return XCP_OK;
  const bool sums = bnpart || fin.acc;
  if (Yb) {   // sums over the final dX: needs the residual input, no skip input, and the BN's statistics
    if (!dRes || dSkip || !sums || !bmean || !binvstd) return XCP_EINVAL;
  } else if (sums && (act != ACT_BNRELU || !bmean || !binvstd)) {
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
  a.fin = fin;
  if (fin.acc) {   // every workgroup of the launch arrives (launch_bwd_lds: 4 waves per workgroup)
    const long waves = (long)N * ((W + RCOLS - 1) / RCOLS) * a.nbands * a.ngroups;
    a.fin.expected = (unsigned)((waves + 3) / 4);
  }
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

// xcp_dw_bwd with the preceding BN's backward finalize folded in (see include/xcp.h)
int xcp_dw_bwd_fin(int dtype, int act, const void* dY, const void* X, const float* Wt, const float* scale,
                   const float* shift, const void* dRes, const void* dSkip, int sOH, int sOW, int sS, int skip_pre,
                   void* dX, float* dWpart, const float* bmean, const float* binvstd, int N, int H, int W, int C, int Cbn,
                   double* acc, unsigned* ticket, const float* gamma, float* alpha, float* bcoef, float* delta,
                   float* dgamma, float* dbeta, int accumulate, hipStream_t stream) {
  if (Cbn <= 0 || Cbn > C || !acc || !ticket || !gamma || !alpha || !bcoef || !delta ||
      (dgamma == nullptr) != (dbeta == nullptr))
    return XCP_EINVAL;
  BnFin f{};
  f.acc = acc;
  f.ticket = ticket;
  f.C = Cbn;
  f.CP = C;
  f.bwd = 1;
  f.count = (double)N * H * W;
  f.gamma = gamma;
  f.o0 = alpha;
  f.o1 = bcoef;
  f.o2 = delta;
  f.mean = bmean;
  f.invstd = binvstd;
  f.dgamma = dgamma;
  f.dbeta = dbeta;
  f.accumulate = accumulate;
  return dw_bwd_impl(dtype, act, dY, X, Wt, scale, shift, dRes, dSkip, sOH, sOW, sS, skip_pre, dX, dWpart, nullptr, bmean,
                     binvstd, nullptr, N, H, W, C, stream, f);
}

int xcp_dw_bwd_resbn(int dtype, int act, const void* dY, const void* X, const float* Wt, const float* scale,
                     const float* shift, const void* dRes, void* dX, float* dWpart, float* bnpart, const float* bmean,
                     const float* binvstd, const void* Yb, int N, int H, int W, int C, hipStream_t stream) {
  return dw_bwd_impl(dtype, act, dY, X, Wt, scale, shift, dRes, nullptr, 0, 0, 1, 0, dX, dWpart, bnpart, bmean, binvstd, Yb,
                     N, H, W, C, stream);
}

}  // extern "C"
