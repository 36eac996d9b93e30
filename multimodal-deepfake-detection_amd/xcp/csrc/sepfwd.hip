// Fused forward of one entry-flow SeparableConv2d: depthwise 3x3 (stride 1, pad 1) followed by the
// 1x1 pointwise conv to 128 channels, with the BatchNorm batch statistics of the pointwise output --
// Xception.py:37-47 (SeparableConv2d.forward = pointwise(conv1(x))) for block1's two units
// (147^2: 64 -> 128, 128 -> 128) and block2's first (74^2: 128 -> 256), whose pointwise GEMMs
// (K = 64 / 128) are HBM-bound.
//
// Unfused, the depthwise output D is written by dw_fwd and read back by the GEMM; here it goes from
// the depthwise FMAs through LDS straight into the MFMAs (D is still written once: the unit's
// backward reads it).  HBM bytes per output pixel: CIN*2 (input) + CIN*2 (D) + 256 (Y), against
// 2*CIN*2 + CIN*2 + 256 for the two kernels.
//
// One 512-thread workgroup per CU walks the rows of a band of one frame (a whole frame when there
// are at least as many frames as CUs), so every input row is fetched once:
//   * LDS holds a sliding window of three activated input rows (all CIN channels, W + 2 pixels with
//     the zero padding); the next rows are loaded into registers two output rows ahead, activated
//     (the previous unit's BatchNorm + ReLU, rounded to bf16 as dw_fwd's staging does) and written
//     over the row that left the window;
//   * an output row is done in two halves of 80 pixels: each lane computes 5 pixels x 2 channels of
//     the depthwise conv from a 3 x 7 window (the fma chain per channel of dw_fwd_w2_kernel, so D is
//     bitwise dw_fwd's) into an LDS tile [80 px][CIN]; wave w then accumulates
//     Y[px][16w .. 16w+15] (and 16(w+8) .. for 256 outputs) += D[px][:] W[..][:]^T with
//     v_mfma_f32_16x16x32_bf16 (the weights of its output channels live in registers; operands and
//     K order as the NT GEMMs, so Y is bitwise theirs) and the D tile is stored with 16-B buffer stores;
//   * the half row's Y goes through LDS (the D tile's space at CIN = 128) so that it leaves as 16-B
//     stores of whole pixel rows (8-B stores of 32-B pieces from the accumulators measured 3-5 %
//     slower); its bf16 values enter per-thread BN sums, written as one partial row per workgroup.
// Every VMEM instruction is issued by every lane (out-of-range loads read a zero line, out-of-range
// buffer stores get an offset past the buffer and are dropped), so the one counted wait per row --
// for the input row loaded two rows ago, with the D and Y stores of the last two rows and the next
// row's loads still in flight -- is exact.
#include "common.h"

namespace {

constexpr int SP_WMAX = 152;                // widest frame (two 80-pixel halves per row)
constexpr int SP_WMAX1 = 78;                // widest frame of the one-half form (COUT = 256)
constexpr int SP_HALF = 80;                 // pixels per half row (5 MFMA blocks)
constexpr int SP_SEG = 5;                   // depthwise outputs per lane
constexpr unsigned SP_OOB = 0x80000000u;
constexpr int SP_REC = 0x7fffffff;
constexpr int SP_DW3 = 0x00020000;

typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef int i32x2 __attribute__((ext_vector_type(2)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef float f2 __attribute__((ext_vector_type(2)));


// prefetch loads by inline asm: hipcc tracks the loads it emits itself and, merging the two register
// sets' states at the row loop's back edge, waited for both sets at every row (one row of look-ahead
// instead of two); these it does not see, so the one counted wait per row is the only one, and
// sp_fence() pins every use of a loaded register after it
// through a buffer resource on the input row (SGPRs) and a 32-bit lane offset: the row's base is
// scalar work, the lane offsets are fixed per thread, and an out-of-range offset (padding columns,
// rows outside the frame via num_records 0) loads zeros -- no 64-bit address arithmetic per load
XCP_DEV u32x4 sp_bload(__amdgpu_buffer_rsrc_t r, int off) {
  u32x4 v;
  asm volatile("buffer_load_dwordx4 %0, %1, %2, 0 offen" : "=v"(v) : "v"(off), "s"(r) : "memory");
  return v;
}

template <int N>
XCP_DEV void sp_fence(u32x4 (&v)[N]) {
#pragma unroll
  for (int i = 0; i < N; ++i) asm volatile("" : "+v"(v[i]));
}

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
  int nbands, bandH;    // row bands per frame (tiles = N * nbands)
};

XCP_DEV void sp_vm_wait(int n) {   // s_waitcnt vmcnt(n), n in [0, 63]
  switch (n < 0 ? 0 : n > 63 ? 63 : n) {
#define SP_VMW(k) case k: asm volatile("s_waitcnt vmcnt(" #k ")" ::: "memory"); break;
    SP_VMW(0) SP_VMW(1) SP_VMW(2) SP_VMW(3) SP_VMW(4) SP_VMW(5) SP_VMW(6) SP_VMW(7)
    SP_VMW(8) SP_VMW(9) SP_VMW(10) SP_VMW(11) SP_VMW(12) SP_VMW(13) SP_VMW(14) SP_VMW(15)
    SP_VMW(16) SP_VMW(17) SP_VMW(18) SP_VMW(19) SP_VMW(20) SP_VMW(21) SP_VMW(22) SP_VMW(23)
    SP_VMW(24) SP_VMW(25) SP_VMW(26) SP_VMW(27) SP_VMW(28) SP_VMW(29) SP_VMW(30) SP_VMW(31)
    SP_VMW(32) SP_VMW(33) SP_VMW(34) SP_VMW(35) SP_VMW(36) SP_VMW(37) SP_VMW(38) SP_VMW(39)
#undef SP_VMW
    default: asm volatile("s_waitcnt vmcnt(40)" ::: "memory"); break;
  }
}

XCP_DEV void sp_barrier() {   // LDS-only workgroup barrier (no vmcnt wait)
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

XCP_DEV float sp_lo(unsigned u) { return __uint_as_float(u << 16); }
XCP_DEV float sp_hi(unsigned u) { return __uint_as_float(u & 0xffff0000u); }
XCP_DEV unsigned sp_pack(float a, float b) { return pk_bf16(a, b); }

// COUT: 128 (block1) or 256 (block2's first unit, whose 74-pixel rows are one half: NHALF = 1)
template <int ACT, int CIN, int COUT, int NHALF>
__global__ __launch_bounds__(512) void sep_fwd_kernel(SepArgs a) {
  constexpr int SP_RPX = (NHALF == 2 ? SP_WMAX : SP_WMAX1) + 2;   // staged pixels per input row (with the padding)
  constexpr int NB = COUT / 128;                  // 16-channel output blocks per wave (w, w + 8)
  constexpr int YC = COUT / 8;                    // 16-B chunks per Y pixel row
  constexpr int S = CIN / 32;                     // K steps of 32
  constexpr int CH = CIN / 8;                     // 16-B chunks per pixel
  constexpr int PB = CIN * 2;                     // bytes per staged pixel
  constexpr int RB = SP_RPX * PB;                 // bytes per staged row slot
  constexpr int DP = PB + 16;                     // D tile pitch (conflict-free b128 fragment reads)
  constexpr int KL = (SP_RPX * CH + 511) / 512;   // input loads per thread per row
  constexpr int KD = (SP_HALF * CH + 511) / 512;  // D stores per thread per half row
  constexpr int LPS = CIN / 2;                    // lanes per depthwise segment (2 channels each)
  constexpr int SPW = 64 / LPS;                   // segments per wave per pass
  constexpr int NPASS = (SP_HALF / SP_SEG) / (8 * SPW);   // passes per half row (16 segments)
  constexpr int YP = COUT * 2 + 16;               // Y staging pitch (the D tile's at CIN = COUT = 128)
  constexpr int KY = (SP_HALF * YC + 511) / 512;  // Y stores per thread per half row
  constexpr bool YSHARE = YP == DP;               // Y staged in the D tile's space
  constexpr int NST = NHALF * (KD + KY);          // stores per output row
  // the per-row wait vmcnt(NST + KL) must retire the oldest register set on every row: on a band's
  // first row only that set's KL-load successor (the other set) and this row's NST stores follow it;
  // on later rows the previous row's NST stores come first and are retired with it
  static_assert(NST + KL <= 39, "counted wait exceeds sp_vm_wait's range");
  __shared__ __attribute__((aligned(16))) char rows[3 * RB];
  __shared__ __attribute__((aligned(16))) char dt[SP_HALF * DP];
  __shared__ __attribute__((aligned(16))) char yown[YSHARE ? 16 : SP_HALF * YP];
  char* const yt = YSHARE ? dt : yown;            // Y half-row staging (after the D tile is stored)
  __shared__ __attribute__((aligned(16))) float stap[9][CIN];   // depthwise taps
  __shared__ __attribute__((aligned(16))) float sprm[2][CIN];   // input BN scale / shift

  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 15, fg = lane >> 4;
  const int H = a.H, W = a.W;
  const int nch = (W + 2) * CH;                   // staged chunks per row
  const __amdgpu_buffer_rsrc_t rD = __builtin_amdgcn_make_buffer_rsrc(a.D, (short)0, SP_REC, SP_DW3);
  const __amdgpu_buffer_rsrc_t rY = __builtin_amdgcn_make_buffer_rsrc(a.Y, (short)0, SP_REC, SP_DW3);

  // ---- this wave's weights in registers; taps and the input BN affine in LDS
  bf16x8 wf[NB][S];
#pragma unroll
  for (int j = 0; j < NB; ++j)
#pragma unroll
    for (int s = 0; s < S; ++s)
      wf[j][s] = *reinterpret_cast<const bf16x8*>(a.pw + (long)((w + 8 * j) * 16 + fr) * CIN + s * 32 + fg * 8);
  for (int c = tid; c < 9 * CIN; c += 512) stap[c / CIN][c % CIN] = a.dwt[c];
  for (int c = tid; c < CIN; c += 512) {
    sprm[0][c] = ACT == ACT_BNRELU ? a.scale[c] : 1.f;
    sprm[1][c] = ACT == ACT_BNRELU ? a.shift[c] : 0.f;
  }
  __syncthreads();
  const int ch = 2 * (lane % LPS);                // depthwise channels ch, ch + 1
  const int q = tid % CH;                         // staging chunk of every load of this thread
  f2 s1[4], s2[4];   // BN sums of channels 8 * (tid % YC) + 0..7
#pragma unroll
  for (int r = 0; r < 4; ++r) s1[r] = s2[r] = f2{0.f, 0.f};

  // input row hh of frame n -> registers (zeros outside the frame and in the padding columns); two
  // register sets, rows two ahead of the one being consumed
  u32x4 rga[KL], rgb[KL];
  int loff[KL];   // byte offset of this thread's chunk k within an input row (SP_OOB: padding / past the row)
#pragma unroll
  for (int k = 0; k < KL; ++k) {
    const int c = tid + 512 * k;
    const int px = c / CH;
    loff[k] = c < nch && px >= 1 && px <= W ? ((px - 1) * CIN + q * 8) * 2 : (int)SP_OOB;
  }
  auto load_row = [&](u32x4 (&rg)[KL], int n, int hh) {
    const bool rok = hh >= 0 && hh < H;   // (uniform)
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<bf16*>(a.X + ((long)n * H + (rok ? hh : 0)) * W * CIN), (short)0, rok ? SP_REC : 0, SP_DW3);
#pragma unroll
    for (int k = 0; k < KL; ++k) rg[k] = sp_bload(rs, loff[k]);
  };
  // registers -> LDS slot of row hh, activated (the padding stays zero)
  auto store_row = [&](u32x4 (&rg)[KL], int hh) {
    sp_fence(rg);
    char* slot = rows + ((hh + 3) % 3) * RB;
#pragma unroll
    for (int k = 0; k < KL; ++k) {
      const int c = tid + 512 * k;
      if (c >= nch) continue;
      const int px = c / CH;
      uint4 u = make_uint4(rg[k][0], rg[k][1], rg[k][2], rg[k][3]);
      if constexpr (ACT != ACT_NONE) {
        if (hh >= 0 && hh < H && px >= 1 && px <= W) {
          unsigned v[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            f2 x = f2{sp_lo(v[e]), sp_hi(v[e])};
            if constexpr (ACT == ACT_BNRELU)
              x = __builtin_elementwise_fma(x, *reinterpret_cast<const f2*>(&sprm[0][q * 8 + 2 * e]),
                                            *reinterpret_cast<const f2*>(&sprm[1][q * 8 + 2 * e]));
            x = __builtin_elementwise_max(x, f2{0.f, 0.f});
            v[e] = sp_pack(x[0], x[1]);
          }
          u = make_uint4(v[0], v[1], v[2], v[3]);
        }
      }
      *reinterpret_cast<uint4*>(slot + px * PB + q * 16) = u;
    }
  };

  const int tiles = a.N * a.nbands;
  for (int tile = xcd_remap(blockIdx.x, gridDim.x); tile < tiles; tile += gridDim.x) {
    const int n = tile / a.nbands, band = tile % a.nbands;
    const int r0 = band * a.bandH, r1 = min(H, r0 + a.bandH);
    // prologue: rows r0-1 .. r0+1 into the window, rows r0+2, r0+3 in flight
    sp_barrier();   // (a previous tile's readers of the window are done)
    for (int hh = r0 - 1; hh <= r0 + 1; ++hh) {
      load_row(rga, n, hh);
      sp_vm_wait(0);
      store_row(rga, hh);
    }
    load_row(rga, n, r0 + 2);
    load_row(rgb, n, r0 + 3);
    sp_barrier();
    auto row = [&](int h, u32x4 (&rg)[KL]) {
      const long prow = ((long)n * H + h) * W;
      const char* rw0 = rows + ((h + 2) % 3) * RB;   // row h-1
      const char* rw1 = rows + ((h + 3) % 3) * RB;   // row h
      const char* rw2 = rows + ((h + 4) % 3) * RB;   // row h+1
#pragma unroll
      for (int hf = 0; hf < NHALF; ++hf) {
        f32x4 acc[5][NB];
#pragma unroll
        for (int b = 0; b < 5; ++b)
#pragma unroll
          for (int j = 0; j < NB; ++j) acc[b][j] = f32x4{0.f, 0.f, 0.f, 0.f};
        // depthwise: segments of 5 pixels, 2 channels per lane, all CIN channels per segment
#pragma unroll 1
        for (int p = 0; p < NPASS; ++p) {
          const int seg = p * 8 * SPW + w * SPW + lane / LPS;
          const int xl = seg * SP_SEG;               // first pixel in the half
          const int x0 = hf * SP_HALF + xl;          // first output pixel (= its window's first staged pixel)
          // (packed pairs: each channel keeps dw_fwd's fma chain in (ky, kx) order)
          f2 tp[9];
#pragma unroll
          for (int t = 0; t < 9; ++t) tp[t] = *reinterpret_cast<const f2*>(&stap[t][ch]);
          f2 win[3][SP_SEG + 2];
#pragma unroll
          for (int k = 0; k < SP_SEG + 2; ++k) {
            const int off = min(x0 + k, W + 1) * PB + ch * 2;
            const unsigned u0 = *reinterpret_cast<const unsigned*>(rw0 + off);
            const unsigned u1 = *reinterpret_cast<const unsigned*>(rw1 + off);
            const unsigned u2 = *reinterpret_cast<const unsigned*>(rw2 + off);
            win[0][k] = f2{sp_lo(u0), sp_hi(u0)};
            win[1][k] = f2{sp_lo(u1), sp_hi(u1)};
            win[2][k] = f2{sp_lo(u2), sp_hi(u2)};
          }
#pragma unroll
          for (int jj = 0; jj < SP_SEG; ++jj) {
            f2 d = f2{0.f, 0.f};
#pragma unroll
            for (int ky = 0; ky < 3; ++ky)
#pragma unroll
              for (int kx = 0; kx < 3; ++kx) d = __builtin_elementwise_fma(win[ky][jj + kx], tp[ky * 3 + kx], d);
            *reinterpret_cast<unsigned*>(dt + (xl + jj) * DP + ch * 2) = x0 + jj < W ? sp_pack(d[0], d[1]) : 0u;
          }
        }
        sp_barrier();   // D tile complete
        // pointwise: acc[b][j] += W[16(w + 8j) + .][:] x D[16b + .][:], K in steps of 32 (the NT GEMMs' order)
#pragma unroll
        for (int b = 0; b < 5; ++b)
#pragma unroll
          for (int s = 0; s < S; ++s) {
            const bf16x8 ad = *reinterpret_cast<const bf16x8*>(dt + (b * 16 + fr) * DP + (s * 32 + fg * 8) * 2);
#pragma unroll
            for (int j = 0; j < NB; ++j) acc[b][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[j][s], ad, acc[b][j], 0, 0, 0);
          }
        // the D half row -> HBM
#pragma unroll
        for (int k = 0; k < KD; ++k) {
          const int c = tid + 512 * k;
          const int pl = min(c / CH, SP_HALF - 1), qq = c % CH;
          const int px = hf * SP_HALF + pl;
          const bool ok = c < SP_HALF * CH && px < W;
          const uint4 v = *reinterpret_cast<const uint4*>(dt + pl * DP + qq * 16);
          const unsigned off = ok ? (unsigned)(((prow + px) * CIN + qq * 8) * 2) : SP_OOB;
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(i32x4, v), rD, (int)off, 0, 0);
        }
        // the half row's Y through LDS: 16-B stores of whole pixel rows, then the BN sums
        if constexpr (YSHARE) sp_barrier();   // every wave is done with the D tile
#pragma unroll
        for (int b = 0; b < 5; ++b)
#pragma unroll
          for (int j = 0; j < NB; ++j)
            *reinterpret_cast<uint2*>(yt + (b * 16 + fr) * YP + ((w + 8 * j) * 16 + 4 * fg) * 2) =
                make_uint2(sp_pack(acc[b][j][0], acc[b][j][1]), sp_pack(acc[b][j][2], acc[b][j][3]));
        sp_barrier();
#pragma unroll
        for (int k = 0; k < KY; ++k) {
          const int c = tid + 512 * k;
          const int pl = min(c / YC, SP_HALF - 1), qq = c % YC;
          const int px = hf * SP_HALF + pl;
          const bool ok = c < SP_HALF * YC && px < W;
          const uint4 v = *reinterpret_cast<const uint4*>(yt + pl * YP + qq * 16);
          const unsigned off = ok ? (unsigned)(((prow + px) * COUT + qq * 8) * 2) : SP_OOB;
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(i32x4, v), rY, (int)off, 0, 0);
          if (ok) {
            const unsigned u4[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const f2 y = f2{sp_lo(u4[r]), sp_hi(u4[r])};
              s1[r] += y;
              s2[r] = __builtin_elementwise_fma(y, y, s2[r]);
            }
          }
        }
        sp_barrier();   // the D tile is free again (and, after the second half, the window row h-1)
      }
      // slide the window: row h+2 (loaded two rows ago into rg) replaces row h-1 and row h+4 goes into
      // rg; issued after row h+2's loads: the stores of rows h-1 and h and the loads of row h+3.  One
      // constant wait leaves this row's stores and row h+3's loads in flight (the previous row's stores,
      // a row old, are retired with it): a single s_waitcnt on every path
      sp_vm_wait(NST + KL);
      store_row(rg, h + 2);
      load_row(rg, n, h + 4);
      sp_barrier();
    };
    for (int h = r0; h < r1; h += 2) {
      row(h, rga);
      if (h + 1 < r1) row(h + 1, rgb);
    }
    sp_vm_wait(0);   // the look-ahead loads past the band land before the next tile reuses their registers
  }
  sp_vm_wait(0);
  // BN partial row of this workgroup: lanes of one channel group (tid % YC) across the wave, then the
  // 8 waves through LDS
  if (a.part) {
    float t[2][8];
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        t[0][2 * r + e] = s1[r][e];
        t[1][2 * r + e] = s2[r][e];
      }
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        if constexpr (YC == 16) t[m][e] += __shfl_xor(t[m][e], 16, 64);
        t[m][e] += __shfl_xor(t[m][e], 32, 64);
      }
    sp_barrier();
    float* red = reinterpret_cast<float*>(rows);   // [8 waves][2][COUT]
    if (lane < YC)
#pragma unroll
      for (int m = 0; m < 2; ++m)
#pragma unroll
        for (int e = 0; e < 8; ++e) red[(w * 2 + m) * COUT + lane * 8 + e] = t[m][e];
    sp_barrier();
    for (int i = tid; i < 2 * COUT; i += 512) {
      float v = 0.f;
#pragma unroll
      for (int ww = 0; ww < 8; ++ww) v += red[ww * 2 * COUT + i];
      a.part[(long)blockIdx.x * 2 * COUT + i] = v;
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

// bands per frame: enough (frame, band) tiles for every CU, bands of at least 8 rows
void sp_bands(int N, int H, int& nb, int& bandH) {
  const int cus = sp_cus();
  nb = N >= cus ? 1 : (cus + N - 1) / N;
  const int maxb = H >= 16 ? H / 8 : 1;
  if (nb > maxb) nb = maxb;
  if (nb < 1) nb = 1;
  bandH = (H + nb - 1) / nb;
  nb = (H + bandH - 1) / bandH;
}

}  // namespace

extern "C" {

// partial-sum rows xcp_sep_fwd writes (one per workgroup); 0: the shape is not supported
int xcp_sep_fwd_parts(int dtype, int N, int H, int W, int CIN, int COUT) {
  // (CIN, COUT) = (64 | 128, 128) up to 152 pixels wide, (128, 256) up to 78
  const bool shape = (COUT == 128 && (CIN == 64 || CIN == 128) && W <= SP_WMAX) ||
                     (COUT == 256 && CIN == 128 && W <= SP_WMAX1);
  if (dtype != XCP_BF16 || !shape || W < 1 || N <= 0 || H <= 0) return 0;
  const long pix = (long)N * H * W;
  if (pix * CIN * 2 > 0x7fffffffL || pix * COUT * 2 > 0x7fffffffL) return 0;   // 32-bit buffer offsets
  int nb, bh;
  sp_bands(N, H, nb, bh);
  const long tiles = (long)N * nb;
  return (int)(tiles < sp_cus() ? tiles : sp_cus());
}

int xcp_sep_fwd(int dtype, int act, const void* X, const float* scale, const float* shift, const float* dwt, const void* pw,
                void* D, void* Y, float* part, int N, int H, int W, int CIN, int COUT, hipStream_t stream) {
  const int grid = xcp_sep_fwd_parts(dtype, N, H, W, CIN, COUT);
  if (grid <= 0) return XCP_EUNSUPPORTED;
  if (act < ACT_NONE || act > ACT_BNRELU || (act == ACT_BNRELU && (!scale || !shift))) return XCP_EINVAL;
  SepArgs a{(const bf16*)X, scale, shift, dwt, (const bf16*)pw, (bf16*)D, (bf16*)Y, part, N, H, W, 1, H};
  sp_bands(N, H, a.nbands, a.bandH);
#define SP_LAUNCH(A, C, O, NH) hipLaunchKernelGGL((sep_fwd_kernel<A, C, O, NH>), dim3(grid), dim3(512), 0, stream, a)
#define SP_ACTS(C, O, NH)                          \
  if (act == ACT_NONE) SP_LAUNCH(ACT_NONE, C, O, NH); \
  else if (act == ACT_RELU) SP_LAUNCH(ACT_RELU, C, O, NH); \
  else SP_LAUNCH(ACT_BNRELU, C, O, NH);
  if (COUT == 256) {
    SP_ACTS(128, 256, 1)
  } else if (CIN == 64) {
    SP_ACTS(64, 128, 2)
  } else {
    SP_ACTS(128, 128, 2)
  }
#undef SP_ACTS
#undef SP_LAUNCH
  return (int)hipGetLastError();
}

}  // extern "C"
