// Stem conv2 (3x3, 32 -> 64, stride 1, pad 0) forward and its input gradient as direct
// MFMA convolutions over LDS-resident row tiles.
//
// Reference op: Xception.conv2 = nn.Conv2d(32, 64, 3, bias=False) (Xception.py:122,
// called at :172) at 149x149 -> 147x147.  Its backward w.r.t. the input is the same
// kind of convolution: dA[h][w][ci] = sum dY[h-2+ky][w-2+kx][co] W[co][8-tap][ci] over the
// zero-padded (pad 2) gradient, i.e. a 64 -> 32 conv with the flipped, transposed kernel.
// The generic implicit-GEMM path (gemm.hip gather modes 2 / 3) re-reads every input chunk
// nine times through L2 and wastes half of its 128-wide N tile on 64 / 32 output channels
// (0.94 / 1.38 ms per call at 256 x 149^2); both directions are HBM-bound
// (~1.07 GB moved per call, ~195 us at 5.5 TB/s).
//
// conv3x3_kernel<CIN, COUT, PAD, TH>: a persistent 512-thread workgroup per CU walks tiles
// of TH output rows (one frame, all COUT channels); the (TH+2) x (IW+2*PAD) input pixels
// of the NEXT tile stream into the second of two LDS buffers by LDS-DMA (16-B chunks
// XOR-swizzled by column through the per-lane source address so the fragment reads below
// are bank-conflict-free at lane offsets fixed per tap column; image padding reads a zero
// line).
// Each wave owns two 16-channel output groups (COUT = 64: waves 0/2 channels 0-31, 1/3
// channels 32-63) and keeps their kernel slice in VGPRs as MFMA A-fragments (2 x 9 x CIN/32
// fragments: 72 VGPRs forward, 144 for the 64-deep dgrad) and walks (output row, 16-pixel
// group) items:
//   D[16 co][16 px] += W[co][tap][32 ci] x In[32 ci][px + tap]   (v_mfma_f32_16x16x32_bf16)
// each B-fragment read from LDS feeds 2 MFMAs (18 / 36 MFMAs per item).  Lanes fg / fg^1 (16 apart)
// swap 8-B pieces of the rounded tile so every lane stores 16 contiguous bytes: one store
// instruction covers 16 consecutive output pixels x 64 B (the whole row segment for
// COUT = 32).  With STATS each workgroup writes its BatchNorm partial sums (sum, sum of
// squares of the stored values) as one row of [wg][2][COUT].  The kernel fragments are
// loaded once per workgroup.
#include "common.h"

namespace {

__device__ __attribute__((aligned(64))) uint4 g_czero[4];

// s_waitcnt vmcnt(n) for a wave-uniform runtime n (the immediate is 6 bits; n >= 16 waits for 15,
// which is stricter)
XCP_DEV void wait_vmcnt_dyn(int n) {
  switch (n) {
#define XCP_VMW(k) \
  case k: asm volatile("s_waitcnt vmcnt(" #k ")" ::: "memory"); break;
    XCP_VMW(0) XCP_VMW(1) XCP_VMW(2) XCP_VMW(3) XCP_VMW(4) XCP_VMW(5) XCP_VMW(6) XCP_VMW(7)
    XCP_VMW(8) XCP_VMW(9) XCP_VMW(10) XCP_VMW(11) XCP_VMW(12) XCP_VMW(13) XCP_VMW(14)
#undef XCP_VMW
    default: asm volatile("s_waitcnt vmcnt(15)" ::: "memory"); break;
  }
}

// In-place BN + ReLU of staged input chunks (ACTIN): LDS accesses by inline asm, since a compiler-visible
// access to LDS an LDS-DMA may still be writing makes hipcc wait for every outstanding vector-memory
// operation (here: the next tile's / row's DMA, issued just before)
typedef unsigned c3u4 __attribute__((ext_vector_type(4)));
typedef unsigned long long u64;
typedef u64 u64x2 __attribute__((ext_vector_type(2)));
XCP_DEV c3u4 c3_rd128(const char* p) {
  c3u4 v;
  asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"((unsigned)(size_t)(const __attribute__((address_space(3))) char*)(p))
               : "memory");
  return v;
}
XCP_DEV void c3_wr128(char* p, c3u4 v) {
  asm volatile("ds_write_b128 %0, %1" :: "v"((unsigned)(size_t)(__attribute__((address_space(3))) char*)(p)), "v"(v)
               : "memory");
}
XCP_DEV u64 ds_read_tr_u64(const char* p) {
  u64 v;
  asm volatile("ds_read_b64_tr_b16 %0, %1"
               : "=v"(v)
               : "v"((unsigned)(size_t)(const __attribute__((address_space(3))) char*)(p))
               : "memory");
  return v;
}
// s_waitcnt lgkmcnt(0) that a chunk's 20 fragment halves depend on (no use is scheduled ahead of it)
XCP_DEV void c3_tr_fence(u64 (&g)[2], u64 (&b)[9][2]) {
  asm volatile("s_waitcnt lgkmcnt(0)"
               : "+v"(g[0]), "+v"(g[1]), "+v"(b[0][0]), "+v"(b[0][1]), "+v"(b[1][0]), "+v"(b[1][1]), "+v"(b[2][0]),
                 "+v"(b[2][1]), "+v"(b[3][0]), "+v"(b[3][1]), "+v"(b[4][0]), "+v"(b[4][1]), "+v"(b[5][0]),
                 "+v"(b[5][1]), "+v"(b[6][0]), "+v"(b[6][1]), "+v"(b[7][0]), "+v"(b[7][1]), "+v"(b[8][0]),
                 "+v"(b[8][1])
               :
               : "memory");
}
// the BN parameters (n <= 64 floats each) into LDS by LDS-DMA from wave 0 (lane i -> word i): a
// compiler-visible global load here makes hipcc drain every in-flight DMA before the main loop's LDS reads
XCP_DEV void c3_load_prm(float* sc, float* sh, const float* isc, const float* ish, int n, int lane) {
  if (lane < n) {
    __builtin_amdgcn_global_load_lds((const void __attribute__((address_space(1)))*)(isc + lane),
                                     (void __attribute__((address_space(3)))*)sc, 4, 0, 0);
    __builtin_amdgcn_global_load_lds((const void __attribute__((address_space(1)))*)(ish + lane),
                                     (void __attribute__((address_space(3)))*)sh, 4, 0, 0);
  }
}
// relu(x * sc + sh) of 8 bf16 (rounded to bf16, as bn_act does); c8: first channel
XCP_DEV c3u4 c3_act(c3u4 v, const float* sc, const float* sh, int c8) {
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const float lo = fmaxf(fmaf(__uint_as_float(v[e] << 16), sc[c8 + 2 * e], sh[c8 + 2 * e]), 0.f);
    const float hi = fmaxf(fmaf(__uint_as_float(v[e] & 0xffff0000u), sc[c8 + 2 * e + 1], sh[c8 + 2 * e + 1]), 0.f);
    v[e] = pk_bf16(lo, hi);
  }
  return v;
}
// activate chunks q = q0, q0 + step, ... < total of an LDS buffer; chunk q holds channels c8(q) .. +7
template <int MAXK, typename C8>
XCP_DEV void c3_act_chunks(char* base, int q0, int step, int total, const float* sc, const float* sh, C8 c8) {
  c3u4 v[MAXK];
#pragma unroll
  for (int k = 0; k < MAXK; ++k) v[k] = c3_rd128(base + min(q0 + k * step, total - 1) * 16);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
  for (int k = 0; k < MAXK; ++k) {
    const int q = q0 + k * step;
    if (q < total) c3_wr128(base + q * 16, c3_act(v[k], sc, sh, c8(q)));
  }
}

// 16-B chunk swizzle of LDS column x (brute-force checked: conflict-free ds_read_b128 for
// 16 consecutive columns at any row offset); depends on x mod 8 only
template <int CIN>
XCP_DEV int cswz(int x) {
  if constexpr (CIN == 32) return (x >> 1) & 3;
  else return x & 7;
}


// ACTIN: X is the raw input of a BatchNorm + ReLU (the stem's conv1 output): each staged tile is
// activated in place, relu(x * isc[c] + ish[c]) rounded to bf16 as bn_act does, before its reads
template <int CIN, int COUT, int PAD, int TH, int MAXIW, bool STATS, int NW, bool PIPE, bool ACTIN = false>
__global__ __launch_bounds__(NW * 64, 8 / NW) void conv3x3_kernel(const bf16* __restrict__ X, const bf16* __restrict__ Wp,
                                                         bf16* __restrict__ Y, float* __restrict__ stats, int N,
                                                         int IH, int IW, const float* __restrict__ isc,
                                                         const float* __restrict__ ish) {
  constexpr int CPP = CIN / 8;                // 16-B chunks per pixel
  constexpr int PB = CPP * 16;                // LDS bytes per pixel
  constexpr int KS = CIN / 32;                // 32-deep MFMA steps per tap
  constexpr int CG = 2;                       // output-channel groups per wave
  constexpr int NCP = COUT / 32;              // channel-group pairs (waves split over them)
  constexpr int BUF = ((TH + 2) * (MAXIW + 2 * PAD) + 16) * PB;   // + slack for junk columns past OW
  constexpr int F3 = 3 * KS;                  // B-fragments per pipeline third (9 x KS per item)
  static_assert(COUT % 32 == 0, "pieces are exchanged between channel-group pairs");
  // (the BN parameters live in the same LDS object as the tiles: with a second object the LDS accesses
  // carry alias scopes, and hipcc then waits for all in-flight DMA before the fragment reads)
  __shared__ __attribute__((aligned(16))) char smem[2 * BUF + (ACTIN ? 8 * CIN : 0)];
  float* const sprm0 = reinterpret_cast<float*>(smem + 2 * BUF);
  float* const sprm1 = sprm0 + CIN;
  const int OH = IH + 2 * PAD - 2, OW = IW + 2 * PAD - 2, LW = IW + 2 * PAD;
  const int tiles_h = (OH + TH - 1) / TH, ntiles = N * tiles_h, G = gridDim.x;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, fr = lane & 15, fg = lane >> 4;
  const int wsc = __builtin_amdgcn_readfirstlane(w);   // wave index, in an SGPR
  const int tile_px = (TH + 2) * LW, total = tile_px * CPP;

  // stage tile t (input rows oh0-PAD .. oh0-PAD+TH+1, zero outside the image) into buffer b
  auto stage = [&](int t, int b) {
    const int n = t / tiles_h, oh0 = (t - n * tiles_h) * TH;
    const bf16* Xn = X + (long)n * IH * IW * CIN;
    for (int q0 = w * 64; q0 < total; q0 += 64 * NW) {
      const int q = q0 + lane;
      if (q < total) {
        const int p = q / CPP, cpos = q - p * CPP;
        const int r = p / LW, x = p - r * LW;
        const int ih = oh0 - PAD + r, iw = x - PAD;
        const int c = cpos ^ cswz<CIN>(PIPE ? x : p);
        const void* src = (ih >= 0 && ih < IH && iw >= 0 && iw < IW)
                              ? (const void*)(Xn + ((long)ih * IW + iw) * CIN + c * 8)
                              : (const void*)g_czero;
        __builtin_amdgcn_global_load_lds((const void __attribute__((address_space(1)))*)src,
                                         (void __attribute__((address_space(3)))*)(smem + b * BUF + q0 * 16), 16,
                                         0, 0);
      }
    }
  };

  int t = blockIdx.x;
  if (t >= ntiles) return;   // uniform, before any barrier
  static_assert(!ACTIN || CIN <= 64, "one DMA lane per channel");
  if constexpr (ACTIN)   // lands with tile t (first wait: vmcnt(0))
    if (wsc == 0) c3_load_prm(sprm0, sprm1, isc, ish, CIN, lane);
  stage(t, 0);

  // ---- kernel fragments, loaded once: wf[cg][tap][ks] = W[co0+cg*16+fr][tap'][ks*32 + fg*8 .. +8]
  // (Wp is [COUT][9][CIN]; PAD == 2 is the flipped kernel: tap' = 8 - tap)
  const int cp = wsc % NCP, co0 = cp * 32;
  bf16x8 wf[CG][9][KS];
#pragma unroll
  for (int cg = 0; cg < CG; ++cg)
#pragma unroll
    for (int tp0 = 0; tp0 < 9; ++tp0)
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        const int tp = PAD ? 8 - tp0 : tp0;
        wf[cg][tp0][ks] =
            *reinterpret_cast<const bf16x8*>(Wp + ((long)(co0 + cg * 16 + fr) * 9 + tp) * CIN + ks * 32 + fg * 8);
      }
  float s1[CG * 4], s2[CG * 4];
#pragma unroll
  for (int q = 0; q < CG * 4; ++q) s1[q] = s2[q] = 0.f;

  const int npg = (OW + 15) / 16;
  // swizzled chunk byte offset of this lane's fragment at tap column kx (item-invariant: the
  // swizzle depends on the column modulo 8 and items start at multiples of 16)
  // (the dgrad, out of registers, swizzles by LDS pixel index instead and computes each
  // read's chunk on the fly -- cswz(x) and cswz(p) are both conflict-free)
  int loff[3][KS];
#pragma unroll
  for (int kx = 0; kx < 3; ++kx)
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) loff[kx][ks] = PIPE ? ((ks * 4 + fg) ^ cswz<CIN>(fr + kx)) << 4 : 0;
  int prev_st = 0;   // global stores this wave issued after the DMA of tile t (one per item)
  for (int k = 0; t < ntiles; ++k, t += G) {
    // tile t landed (this wave's DMA; the previous tile's stores, issued after it, may stay in
    // flight) -> for every wave.  (__syncthreads would wait for those stores too: vmcnt(0).)
    wait_vmcnt_dyn(prev_st);
    lds_barrier();
    if constexpr (ACTIN) {   // (rows past the image turn from zero into junk that only rows past OH read)
      // before the next tile's DMA is issued: no LDS-DMA is in flight while the tile is rewritten
      constexpr int MAXK = ((TH + 2) * MAXIW * CPP + NW * 64 - 1) / (NW * 64);
      c3_act_chunks<MAXK>(smem + (k & 1) * BUF, tid, NW * 64, total, sprm0, sprm1, [&](int q) {
        const int p = q / CPP, cpos = q - p * CPP;
        return (cpos ^ cswz<CIN>(PIPE ? p % LW : p)) * 8;
      });
      lds_barrier();
    }
    if (t + G < ntiles) stage(t + G, (k + 1) & 1);   // streams in under this tile's MFMAs
    const char* sb = smem + (k & 1) * BUF;
    const int n = t / tiles_h, oh0 = (t - n * tiles_h) * TH;
    // this wave's items (row-major over (row, 16-pixel group)), software-pipelined over three
    // thirds of the 9 x KS B-fragments: the reads of the next third fly under the MFMAs of
    // the current one (two thirds live at a time)
    const int it0 = wsc / NCP, its = NW / NCP;
    const int rows_here = min(TH, OH - oh0);
    const int nit = it0 < rows_here * npg ? (rows_here * npg - it0 + its - 1) / its : 0;
    // fragment f (tap f / KS, 32-channel step f % KS) of item it: the item's lane base, the
    // tap's pixel offset and the lane's swizzled chunk (loff); columns past OW read junk (in
    // the buffer's slack) that is never stored
    auto frag = [&](int it, int f) {
      const int r = it / npg, pg = it - r * npg;
      const int tp = f / KS, ks = f - tp * KS;
      if constexpr (PIPE) {
        const char* base = sb + (r * LW + pg * 16 + fr) * PB;
        return *reinterpret_cast<const bf16x8*>(base + ((tp / 3) * LW + tp % 3) * PB + loff[tp % 3][ks]);
      } else {
        const int p = (r + tp / 3) * LW + pg * 16 + fr + tp % 3;
        return *reinterpret_cast<const bf16x8*>(sb + p * PB + (((ks * 4 + fg) ^ cswz<CIN>(p)) << 4));
      }
    };
    bf16x8 bA[F3], bB[F3], bC[F3];
    auto load3 = [&](bf16x8 (&b)[F3], int it, int part) {
#pragma unroll
      for (int f = 0; f < F3; ++f) b[f] = frag(it, part * F3 + f);
    };
    auto mfma3 = [&](f32x4 (&acc)[CG], const bf16x8 (&b)[F3], int part) {
#pragma unroll
      for (int f = 0; f < F3; ++f) {
        const int ff = part * F3 + f;
#pragma unroll
        for (int cg = 0; cg < CG; ++cg)
          acc[cg] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[cg][ff / KS][ff % KS], b[f], acc[cg], 0, 0, 0);
      }
    };
    if (PIPE && nit > 0) load3(bA, it0, 0);
    for (int j = 0; j < nit; ++j) {
      const int it = it0 + j * its;
      const int r = it / npg, pg = it - r * npg;
      const int oh = oh0 + r;
      f32x4 acc[CG];
#pragma unroll
      for (int cg = 0; cg < CG; ++cg) acc[cg] = f32x4{0.f, 0.f, 0.f, 0.f};
      if constexpr (PIPE) {   // thirds rotate: the next third's reads fly under this third's MFMAs
        load3(bB, it, 1);
        __builtin_amdgcn_sched_barrier(0);
        mfma3(acc, bA, 0);
        __builtin_amdgcn_sched_barrier(0);
        load3(bC, it, 2);
        __builtin_amdgcn_sched_barrier(0);
        mfma3(acc, bB, 1);
        __builtin_amdgcn_sched_barrier(0);
        if (j + 1 < nit) load3(bA, it + its, 0);
        __builtin_amdgcn_sched_barrier(0);
        mfma3(acc, bC, 2);
      } else {                // every read of the item ahead of its MFMAs (fewer live registers)
        load3(bA, it, 0);
        load3(bB, it, 1);
        load3(bC, it, 2);
        __builtin_amdgcn_sched_barrier(0);
        mfma3(acc, bA, 0);
        mfma3(acc, bB, 1);
        mfma3(acc, bC, 2);
      }
      // acc[cg][i] = out[pixel pg*16 + fr][co = co0 + cg*16 + 4fg + i]
      const int ow = pg * 16 + fr;
      const bool ok = ow < OW;
      const bool odd = fg & 1;
      uint2 pc[2];
#pragma unroll
      for (int cg = 0; cg < CG; ++cg) {
        pc[cg] = make_uint2(pk_bf16(acc[cg][0], acc[cg][1]), pk_bf16(acc[cg][2], acc[cg][3]));
        const bf16x4 v = __builtin_bit_cast(bf16x4, pc[cg]);
        if (STATS && ok) {
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const float f = (float)v[i];
            s1[cg * 4 + i] += f;
            s2[cg * 4 + i] = fmaf(f, f, s2[cg * 4 + i]);
          }
        }
      }
      const uint2 snd = odd ? pc[0] : pc[1];
      uint2 rc;
      rc.x = __shfl_xor(snd.x, 16, 64);
      rc.y = __shfl_xor(snd.y, 16, 64);
      const uint4 d = odd ? make_uint4(rc.x, rc.y, pc[1].x, pc[1].y) : make_uint4(pc[0].x, pc[0].y, rc.x, rc.y);
      bf16* ypix = Y + (((long)n * OH + oh) * OW + ow) * COUT + co0 + (odd ? 16 + 4 * (fg - 1) : 4 * fg);
      if (ok) *reinterpret_cast<uint4*>(ypix) = d;
    }
    prev_st = nit;
    lds_barrier();   // every wave is done reading buffer k&1 before it is restaged (LDS only)
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

  if constexpr (STATS) {
    // reduce over the 16 pixel lanes (xor 1..8), then over the waves in LDS
#pragma unroll
    for (int q = 0; q < CG * 4; ++q) {
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) {
        s1[q] += __shfl_xor(s1[q], o, 64);
        s2[q] += __shfl_xor(s2[q], o, 64);
      }
    }
    float* red = reinterpret_cast<float*>(smem);   // [NW / NCP wave rows][2][COUT]; no tile is staged any more
    if (fr == 0) {
#pragma unroll
      for (int cg = 0; cg < CG; ++cg)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          red[((w / NCP) * 2 + 0) * COUT + co0 + cg * 16 + 4 * fg + i] = s1[cg * 4 + i];
          red[((w / NCP) * 2 + 1) * COUT + co0 + cg * 16 + 4 * fg + i] = s2[cg * 4 + i];
        }
    }
    __syncthreads();
    if (tid < 2 * COUT) {
      const int kk = tid / COUT, co = tid - kk * COUT;
      float tot = 0.f;
#pragma unroll
      for (int q = 0; q < NW / NCP; ++q) tot += red[(q * 2 + kk) * COUT + co];
      stats[((long)blockIdx.x * 2 + kk) * COUT + co] = tot;
    }
  }
}

// ---------------------------------------------------------------------------------
// Stem conv2 weight gradient: dW[co][tap][ci] = sum over output pixels p of
// dY[p][co] * X[p + tap][ci]  (tap = kh*3 + kw; 64 x 288 outputs, 2 * 64 * 288 flops per
// output pixel), the reduction running over all N * 147 * 147 pixels.  The generic path
// (gemm.hip gemm_tn_kernel, im2col gather mode 2) took 1.0 ms per call at 256 x 149^2:
// every X chunk is gathered nine times and the output tile is half empty.
//
// conv3x3_wgrad_kernel: one 512-thread workgroup per band of output rows of one frame
// (bands sized so the grid is about one workgroup per CU) slides down its band one output
// row at a time.  LDS holds a 3-slot ring of dY rows ([160 px][64 co], 16-B chunks
// XOR-swizzled by pixel & 7) and a 5-slot ring of X rows ([192 px][32 ci], chunks swizzled
// by bit 2 of the pixel); both are filled by LDS-DMA two rows ahead (4 KB-instructions per
// wave per row, counted vmcnt), pixels past the row read a zero line.  Wave w owns the
// 16 x 16 (co, ci) block (w >> 1, w & 1) for all nine taps (9 accumulators): per 32-pixel
// chunk it reads one transposed dY fragment (ds_read_b64_tr_b16, reused by the 9 taps) and
// nine shifted X fragments, 9 MFMAs (v_mfma_f32_16x16x32_bf16 with the pixels as the
// reduction index).  Each workgroup writes one fp32 slab P[wg][64][288]; the slabs are
// summed by colreduce.
constexpr int WG_GPX = 160, WG_APX = 192;                  // pixels per dY / X ring slot
constexpr int WG_GSLOT = WG_GPX * 128, WG_ASLOT = WG_APX * 64;
constexpr int WG_GI = WG_GSLOT / 1024, WG_AI = WG_ASLOT / 1024;   // 1-KB DMA instructions per row: 20, 12
static_assert((WG_GI + WG_AI) % 8 == 0, "uniform DMA count per wave");
constexpr int WG_PER_WAVE = (WG_GI + WG_AI) / 8;            // 4

// ACTIN: X is the raw input of a BatchNorm + ReLU (isc / ish), activated in place as each row lands
template <bool ACTIN>
__global__ __launch_bounds__(512, 1) void conv3x3_wgrad_kernel(const bf16* __restrict__ dY, const bf16* __restrict__ X,
                                                               float* __restrict__ P, int N, int IH, int IW, int nb,
                                                               int RB, const float* __restrict__ isc,
                                                               const float* __restrict__ ish) {
  // (BN parameters inside the ring's LDS object: see conv3x3_kernel)
  __shared__ __attribute__((aligned(16))) char smem[3 * WG_GSLOT + 5 * WG_ASLOT + (ACTIN ? 256 : 0)];
  float* const sprm0 = reinterpret_cast<float*>(smem + 3 * WG_GSLOT + 5 * WG_ASLOT);
  float* const sprm1 = sprm0 + 32;
  char* gs = smem;
  char* as = smem + 3 * WG_GSLOT;
  const int OH = IH - 2, OW = IW - 2;
  const int n = blockIdx.x / nb, band = blockIdx.x - n * nb;
  const int r0 = band * RB, r1 = min(OH, r0 + RB);
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, fr = lane & 15, fg = lane >> 4;
  const int wsc = __builtin_amdgcn_readfirstlane(w);
  const bf16* Gn = dY + (long)n * OH * OW * 64;
  const bf16* Xn = X + (long)n * IH * IW * 32;
  auto dma = [](const void* src, char* dst) {
    __builtin_amdgcn_global_load_lds((const void __attribute__((address_space(1)))*)src,
                                     (void __attribute__((address_space(3)))*)dst, 16, 0, 0);
  };
  // DMA instruction j of a dY row (j < WG_GI) or of an X row
  auto g_instr = [&](int row, int j) {
    const int q = j * 64 + lane, px = q >> 3, c = (q & 7) ^ (px & 7);
    const void* src = px < OW ? (const void*)(Gn + ((long)row * OW + px) * 64 + c * 8) : (const void*)g_czero;
    dma(src, gs + (row % 3) * WG_GSLOT + j * 1024);
  };
  auto a_instr = [&](int row, int j) {
    const int q = j * 64 + lane, px = q >> 2, c = (q & 3) ^ (((px >> 2) & 1) << 1);
    const void* src = px < IW ? (const void*)(Xn + ((long)row * IW + px) * 32 + c * 8) : (const void*)g_czero;
    dma(src, as + (row % 5) * WG_ASLOT + j * 1024);
  };
  // loads of step oh: dY row oh and X row oh + 2 (4 instructions per wave)
  auto issue_step = [&](int oh) {
#pragma unroll
    for (int i = 0; i < WG_PER_WAVE; ++i) {
      const int j = wsc * WG_PER_WAVE + i;
      if (j < WG_GI) g_instr(oh, j);
      else a_instr(oh + 2, j - WG_GI);
    }
  };
  if (r0 >= r1) return;   // uniform
  if constexpr (ACTIN)   // issued before the rows: complete at the first step's wait
    if (wsc == 0) c3_load_prm(sprm0, sprm1, isc, ish, 32, lane);
  // X row of ring slot row % 5 activated in place (pixels past IW turn into junk that meets only the
  // zero dY past OW)
  auto act_row = [&](int row) {
    c3_act_chunks<(WG_APX * 4 + 511) / 512>(as + (row % 5) * WG_ASLOT, tid, 512, WG_APX * 4, sprm0, sprm1,
                                            [](int q) { return ((q & 3) ^ ((((q >> 2) >> 2) & 1) << 1)) * 8; });
  };
  // prologue: dY row r0 and X rows r0, r0 + 1, r0 + 2 (56 instructions, 7 per wave), then step r0 + 1
#pragma unroll
  for (int i = 0; i < 7; ++i) {
    const int j = wsc * 7 + i;
    if (j < WG_GI) g_instr(r0, j);
    else a_instr(r0 + (j - WG_GI) / WG_AI, (j - WG_GI) % WG_AI);
  }
  if (r0 + 1 < r1) issue_step(r0 + 1);

  const int cb = wsc >> 1, bb = wsc & 1;   // co block (16), ci block (16)
  const int q4 = fr >> 2, p4 = fr & 3;
  // per-lane byte offsets inside a slot: dY fragment rows 4fg + q4 (+16), columns 16cb + 4p4;
  // X fragment columns 16bb + 4p4 at pixel rows 4fg + q4 (+16) + chunk + kw
  const int gch = 2 * cb + (p4 >> 1), ach = 2 * bb + (p4 >> 1), sub = (p4 & 1) * 8;
  f32x4 acc[9];
#pragma unroll
  for (int t = 0; t < 9; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int nch = (OW + 31) / 32;
  for (int oh = r0; oh < r1; ++oh) {
    if (oh + 1 < r1) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    lds_barrier();   // (not __syncthreads: that would also drain the next row's DMA)
    if (oh + 2 < r1) issue_step(oh + 2);
    if constexpr (ACTIN) {   // the X row that landed for this step (at the first step all three)
      if (oh == r0) {
        act_row(r0);
        act_row(r0 + 1);
      }
      act_row(oh + 2);
      lds_barrier();
    }
    const char* gslot = gs + (oh % 3) * WG_GSLOT;
    const char* a0 = as + (oh % 5) * WG_ASLOT;
    const char* a1 = as + ((oh + 1) % 5) * WG_ASLOT;
    const char* a2 = as + ((oh + 2) % 5) * WG_ASLOT;
    const char* arow[3] = {a0, a1, a2};
    // fragments of chunk ch: the transposed dY fragment (g) and the nine shifted X fragments (b), each
    // two 64-bit halves.  Transposed reads by inline asm: hipcc waits vmcnt(0) before every
    // ds_read_tr builtin while any LDS-DMA is in flight (here: the next two rows, drained each row);
    // the counted vmcnt + barrier above orders them, c3_tr_fence retires them before their use.
    auto rd = [&](int ch, u64 (&g)[2], u64 (&b)[9][2]) {
      const int pb = ch * 32 + 4 * fg + q4;
      g[0] = ds_read_tr_u64(gslot + pb * 128 + ((gch ^ (pb & 7)) << 4) + sub);
      g[1] = ds_read_tr_u64(gslot + (pb + 16) * 128 + ((gch ^ ((pb + 16) & 7)) << 4) + sub);
#pragma unroll
      for (int kh = 0; kh < 3; ++kh)
#pragma unroll
        for (int kw = 0; kw < 3; ++kw) {
          const int plo = pb + kw, phi = pb + kw + 16;
          b[kh * 3 + kw][0] = ds_read_tr_u64(arow[kh] + plo * 64 + ((ach ^ (((plo >> 2) & 1) << 1)) << 4) + sub);
          b[kh * 3 + kw][1] = ds_read_tr_u64(arow[kh] + phi * 64 + ((ach ^ (((phi >> 2) & 1) << 1)) << 4) + sub);
        }
    };
    auto mma = [&](const u64 (&g)[2], const u64 (&b)[9][2]) {
      const bf16x8 A = __builtin_bit_cast(bf16x8, u64x2{g[0], g[1]});
#pragma unroll
      for (int t = 0; t < 9; ++t)
        acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A, __builtin_bit_cast(bf16x8, u64x2{b[t][0], b[t][1]}), acc[t],
                                                         0, 0, 0);
    };
    // two register sets: chunk ch + 1's reads fly under chunk ch's MFMAs
    u64 gA[2], bA[9][2], gB[2], bB[9][2];
    rd(0, gA, bA);
    for (int ch = 0; ch < nch; ch += 2) {
      c3_tr_fence(gA, bA);
      if (ch + 1 < nch) rd(ch + 1, gB, bB);
      mma(gA, bA);
      if (ch + 1 >= nch) break;
      c3_tr_fence(gB, bB);
      if (ch + 2 < nch) rd(ch + 2, gA, bA);
      mma(gB, bB);
    }
  }
  // acc[t][r] = dW[co = 16cb + 4fg + r][tap t][ci = 16bb + fr]
  float* Pb = P + (long)blockIdx.x * 64 * 288;
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) Pb[(16 * cb + 4 * fg + r) * 288 + t * 32 + 16 * bb + fr] = acc[t][r];
}

// Shifted-gradient form (conv3x3_wgrad_s_kernel<.., 1>, the default; XCP_CONV3_WGRAD=0 runs the kernel above).
// The kernel above reads, per 32-pixel chunk, one dY fragment and nine X fragments (one per tap) for
// 9 MFMAs: 20 transposed LDS reads (10 KB per wave) per 9 MFMAs.
// Indexing the reduction by the INPUT pixel q = ow + kw instead,
//   dW[co][kh, kw][ci] = sum_oh sum_q dY[oh][q - kw][co] * X[oh + kh][q][ci],
// the nine taps need three X fragments (one per input row kh, unshifted) and three dY fragments (one
// per column shift kw, shared by the three rows): 12 reads per 9 MFMAs.  The dY ring slot holds pixel
// p at position p + 2 (positions 0, 1 and past OW + 1 are zero lines), so q - kw never leaves the slot
// and every q >= OW + kw meets a zero gradient (also the junk an ACTIN row holds past IW).  CP = 2:
// a wave owns two co blocks for the nine taps (6 dY + 3 X fragments per 18 MFMAs) and every other
// chunk; the two chunk halves are summed through LDS at the end (one slab per workgroup either way).
constexpr int WS_GPX = 176, WS_APX = 160;                   // positions per dY / X ring slot
constexpr int WS_GSLOT = WS_GPX * 128, WS_ASLOT = WS_APX * 64;
constexpr int WS_GI = WS_GSLOT / 1024, WS_AI = WS_ASLOT / 1024;   // 22, 10
static_assert((WS_GI + WS_AI) == 32, "4 DMA instructions per wave per row");
constexpr int WS_LDS = 3 * WS_GSLOT + 5 * WS_ASLOT;
static_assert(WS_LDS >= 4 * 18 * 4 * 64 * 4, "the CP = 2 chunk-half reduction fits in the ring");

template <bool ACTIN, int CP>
__global__ __launch_bounds__(512, 1) void conv3x3_wgrad_s_kernel(const bf16* __restrict__ dY, const bf16* __restrict__ X,
                                                                 float* __restrict__ P, int N, int IH, int IW, int nb,
                                                                 int RB, const float* __restrict__ isc,
                                                                 const float* __restrict__ ish) {
  __shared__ __attribute__((aligned(16))) char smem[WS_LDS + (ACTIN ? 256 : 0)];
  float* const sprm0 = reinterpret_cast<float*>(smem + WS_LDS);
  float* const sprm1 = sprm0 + 32;
  char* gs = smem;
  char* as = smem + 3 * WS_GSLOT;
  const int OH = IH - 2, OW = IW - 2;
  const int n = blockIdx.x / nb, band = blockIdx.x - n * nb;
  const int r0 = band * RB, r1 = min(OH, r0 + RB);
  const int tid = threadIdx.x, lane = tid & 63, fr = lane & 15, fg = lane >> 4;
  const int wsc = __builtin_amdgcn_readfirstlane(tid >> 6);
  const bf16* Gn = dY + (long)n * OH * OW * 64;
  const bf16* Xn = X + (long)n * IH * IW * 32;
  auto dma = [](const void* src, char* dst) {
    __builtin_amdgcn_global_load_lds((const void __attribute__((address_space(1)))*)src,
                                     (void __attribute__((address_space(3)))*)dst, 16, 0, 0);
  };
  auto g_instr = [&](int row, int j) {   // dY row: position pos holds pixel pos - 2
    const int q = j * 64 + lane, pos = q >> 3, c = (q & 7) ^ (pos & 7), px = pos - 2;
    const void* src = px >= 0 && px < OW ? (const void*)(Gn + ((long)row * OW + px) * 64 + c * 8) : (const void*)g_czero;
    dma(src, gs + (row % 3) * WS_GSLOT + j * 1024);
  };
  auto a_instr = [&](int row, int j) {
    const int q = j * 64 + lane, px = q >> 2, c = (q & 3) ^ (((px >> 2) & 1) << 1);
    const void* src = px < IW ? (const void*)(Xn + ((long)row * IW + px) * 32 + c * 8) : (const void*)g_czero;
    dma(src, as + (row % 5) * WS_ASLOT + j * 1024);
  };
  auto issue_step = [&](int oh) {   // dY row oh, X row oh + 2: 4 instructions per wave
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int j = wsc * 4 + i;
      if (j < WS_GI) g_instr(oh, j);
      else a_instr(oh + 2, j - WS_GI);
    }
  };
  if (r0 >= r1) return;   // uniform
  if constexpr (ACTIN)
    if (wsc == 0) c3_load_prm(sprm0, sprm1, isc, ish, 32, lane);
  auto act_row = [&](int row) {
    c3_act_chunks<(WS_APX * 4 + 511) / 512>(as + (row % 5) * WS_ASLOT, tid, 512, WS_APX * 4, sprm0, sprm1,
                                            [](int q) { return ((q & 3) ^ ((((q >> 2) >> 2) & 1) << 1)) * 8; });
  };
  // prologue: dY row r0 and X rows r0 .. r0 + 2 (52 instructions over 7 per wave), then step r0 + 1
#pragma unroll
  for (int i = 0; i < 7; ++i) {
    const int j = wsc * 7 + i;
    if (j < WS_GI) g_instr(r0, j);
    else if (j < WS_GI + 3 * WS_AI) a_instr(r0 + (j - WS_GI) / WS_AI, (j - WS_GI) % WS_AI);
  }
  if (r0 + 1 < r1) issue_step(r0 + 1);

  // CP = 1: wave = (co block, ci block), every chunk; CP = 2: wave = (co pair, ci block, chunk half)
  const int bb = CP == 1 ? (wsc & 1) : ((wsc >> 1) & 1);
  const int cb0 = CP == 1 ? (wsc >> 1) : 2 * (wsc >> 2);
  const int h = CP == 1 ? 0 : (wsc & 1);
  const int q4 = fr >> 2, p4 = fr & 3, sub = (p4 & 1) * 8;
  const int ach = 2 * bb + (p4 >> 1);
  f32x4 acc[CP][9];
#pragma unroll
  for (int c = 0; c < CP; ++c)
#pragma unroll
    for (int t = 0; t < 9; ++t) acc[c][t] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int nch = (IW + 31) / 32;
  for (int oh = r0; oh < r1; ++oh) {
    if (oh + 1 < r1) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    lds_barrier();
    if (oh + 2 < r1) issue_step(oh + 2);
    if constexpr (ACTIN) {
      if (oh == r0) {
        act_row(r0);
        act_row(r0 + 1);
      }
      act_row(oh + 2);
      lds_barrier();
    }
    const char* gslot = gs + (oh % 3) * WS_GSLOT;
    const char* arow[3] = {as + (oh % 5) * WS_ASLOT, as + ((oh + 1) % 5) * WS_ASLOT, as + ((oh + 2) % 5) * WS_ASLOT};
    // chunk ch: dY fragments g[c][kw] (co block cb0 + c, pixels q - kw) and X fragments x[kh] (row oh + kh)
    auto rd = [&](int ch, u64 (&g)[CP][3][2], u64 (&x)[3][2]) {
      const int pb = ch * 32 + 4 * fg + q4;
#pragma unroll
      for (int kh = 0; kh < 3; ++kh) {
        x[kh][0] = ds_read_tr_u64(arow[kh] + pb * 64 + ((ach ^ (((pb >> 2) & 1) << 1)) << 4) + sub);
        x[kh][1] = ds_read_tr_u64(arow[kh] + (pb + 16) * 64 + ((ach ^ ((((pb + 16) >> 2) & 1) << 1)) << 4) + sub);
      }
#pragma unroll
      for (int c = 0; c < CP; ++c) {
        const int gch = 2 * (cb0 + c) + (p4 >> 1);
#pragma unroll
        for (int kw = 0; kw < 3; ++kw) {
          const int lo = pb - kw + 2, hi = lo + 16;
          g[c][kw][0] = ds_read_tr_u64(gslot + lo * 128 + ((gch ^ (lo & 7)) << 4) + sub);
          g[c][kw][1] = ds_read_tr_u64(gslot + hi * 128 + ((gch ^ (hi & 7)) << 4) + sub);
        }
      }
    };
    // retire the chunk's reads: the wait, then every fragment pinned after it (volatile asm keeps the order)
    auto fence = [&](u64 (&g)[CP][3][2], u64 (&x)[3][2]) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
      for (int kh = 0; kh < 3; ++kh) asm volatile("" : "+v"(x[kh][0]), "+v"(x[kh][1]));
#pragma unroll
      for (int c = 0; c < CP; ++c)
#pragma unroll
        for (int kw = 0; kw < 3; ++kw) asm volatile("" : "+v"(g[c][kw][0]), "+v"(g[c][kw][1]));
    };
    auto mma = [&](const u64 (&g)[CP][3][2], const u64 (&x)[3][2]) {
#pragma unroll
      for (int c = 0; c < CP; ++c)
#pragma unroll
        for (int kh = 0; kh < 3; ++kh)
#pragma unroll
          for (int kw = 0; kw < 3; ++kw)
            acc[c][kh * 3 + kw] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                __builtin_bit_cast(bf16x8, u64x2{g[c][kw][0], g[c][kw][1]}),
                __builtin_bit_cast(bf16x8, u64x2{x[kh][0], x[kh][1]}), acc[c][kh * 3 + kw], 0, 0, 0);
    };
    // two register sets: the next chunk's reads fly under this chunk's MFMAs
    u64 gA[CP][3][2], xA[3][2], gB[CP][3][2], xB[3][2];
    if (h < nch) rd(h, gA, xA);
    for (int ch = h; ch < nch; ch += 2 * CP) {
      fence(gA, xA);
      if (ch + CP < nch) rd(ch + CP, gB, xB);
      mma(gA, xA);
      if (ch + CP >= nch) break;
      fence(gB, xB);
      if (ch + 2 * CP < nch) rd(ch + 2 * CP, gA, xA);
      mma(gB, xB);
    }
  }
  // acc[c][t][r] = dW[co = 16 (cb0 + c) + 4 fg + r][tap t][ci = 16 bb + fr]
  float* Pb = P + (long)blockIdx.x * 64 * 288;
  if constexpr (CP == 2) {   // the odd-chunk waves hand their sums to the even-chunk waves through the ring
    __syncthreads();
    float* red = reinterpret_cast<float*>(smem) + (wsc >> 1) * (18 * 4 * 64);
    if (h == 1) {
#pragma unroll
      for (int c = 0; c < 2; ++c)
#pragma unroll
        for (int t = 0; t < 9; ++t)
#pragma unroll
          for (int r = 0; r < 4; ++r) red[((c * 9 + t) * 4 + r) * 64 + lane] = acc[c][t][r];
    }
    __syncthreads();
    if (h == 1) return;
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int t = 0; t < 9; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[c][t][r] += red[((c * 9 + t) * 4 + r) * 64 + lane];
  }
#pragma unroll
  for (int c = 0; c < CP; ++c)
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        Pb[(16 * (cb0 + c) + 4 * fg + r) * 288 + t * 32 + 16 * bb + fr] = acc[c][t][r];
}

// XCP_CONV3_WGRAD: 0 = conv3x3_wgrad_kernel, 1 (default) = the shifted form, one co block per wave, 2 = two
// co blocks per wave (read per call: the tests compare the forms in one process).  Alone at 256 x 149^2:
// 392 / 345 / 343 us with the slab reduction; in the step form 1 is +0.35 % over form 0 and form 2 +0.1 %:
// at 225-238 VGPRs form 2 leaves no room on its SIMDs for the BN1 sums (chanred, 138 VGPRs) that run beside
// it, form 1 at 169 does (profiles/r06_conv3_wgrad_ab.txt)
int conv3_wgrad_form() {
  const char* e = getenv("XCP_CONV3_WGRAD");
  return e && (e[0] == '0' || e[0] == '2') ? e[0] - '0' : 1;
}

// bands per frame for the weight-gradient grid: about one workgroup per CU, >= 8 rows a band

// rows per tile and the widest input each direction supports (two LDS tile buffers of 57 /
// 77 KB per workgroup, one workgroup per CU); the Xception stem at 299^2 is 149 -> 147
// (forward), 147 -> 149 (dgrad)
constexpr int TH_FWD = 4, TH_DGRAD = 2, MAXIW_FWD = 149, MAXIW_DGRAD = 147;
// waves per workgroup (two per SIMD); the 64-deep dgrad keeps 144 VGPRs of kernel fragments
// and has no room for the rotating read pipeline
constexpr int NW_FWD = 8, NW_DGRAD = 8;
// XCP_CONV3_FWD_2WG=1: the forward as two workgroups of 4 waves per CU on 2-row tiles (2 x 78 KB of LDS):
// twice the tiles in flight per CU (A/B)
constexpr int TH_FWD2 = 2, NW_FWD2 = 4;
bool conv3_fwd_2wg() {   // (read per call: a test compares both forms in one process)
  const char* e = getenv("XCP_CONV3_FWD_2WG");
  return e && e[0] == '1';
}


int conv3_cus() {
  static const int cus = [] {
    int d = 0, n = 0;
    if (hipGetDevice(&d) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, d) != hipSuccess)
      n = 0;
    return n > 0 ? n : 256;
  }();
  return cus;
}

// weight-gradient grid: bands of output rows per frame, about one workgroup per CU and
// at least 8 rows a band
void wgrad_bands(int N, int OH, int& nb, int& rb) {
  nb = (conv3_cus() + N - 1) / N;
  if (nb > OH / 8) nb = OH / 8;
  if (nb < 1) nb = 1;
  rb = (OH + nb - 1) / nb;
  nb = (OH + rb - 1) / rb;
}

}  // namespace


extern "C" {

// persistent workgroups (= rows of the stats partial array) of xcp_conv3x3; 0 when the
// width is unsupported
int xcp_conv3x3_parts(int mode, int N, int IH, int IW) {
  if (IW > (mode == 0 ? MAXIW_FWD : MAXIW_DGRAD)) return 0;
  const int OH = mode == 0 ? IH - 2 : IH + 2;
  const bool two = mode == 0 && conv3_fwd_2wg();
  const int th = mode == 0 ? (two ? TH_FWD2 : TH_FWD) : TH_DGRAD;
  const int tiles = N * ((OH + th - 1) / th), cap = (two ? 2 : 1) * conv3_cus();
  return tiles < cap ? tiles : cap;
}

// mode 0: Y[N][IH-2][IW-2][64] = conv3x3(X[N][IH][IW][32], W[64][9][32]) (+ BN partial sums)
// mode 1: Y[N][IH+2][IW+2][32] = input gradient of that conv from X = dY[N][IH][IW][64],
//         W = the forward kernel transposed to [32][9][64] (flipped inside).  bf16 only.
int xcp_conv3x3(int mode, const void* X, const void* W, void* Y, float* stats, int N, int IH, int IW,
                const float* in_scale, const float* in_shift, hipStream_t st) {
  if (N <= 0) return XCP_OK;
  if (IH < 3 || IW < 3 || (mode != 0 && mode != 1) || (mode == 1 && stats)) return XCP_EINVAL;
  if ((in_scale != nullptr) != (in_shift != nullptr) || (mode == 1 && in_scale)) return XCP_EINVAL;
  if (IW > (mode == 0 ? MAXIW_FWD : MAXIW_DGRAD)) return XCP_EUNSUPPORTED;
  const dim3 grid((unsigned)xcp_conv3x3_parts(mode, N, IH, IW));
  const bf16 *x = (const bf16*)X, *w = (const bf16*)W;
  bf16* y = (bf16*)Y;
#define XCP_C3F(TH, NW, STATS, ACT)                                                                                  \
  hipLaunchKernelGGL((conv3x3_kernel<32, 64, 0, TH, MAXIW_FWD, STATS, NW, true, ACT>), grid, dim3(64 * NW), 0, st, x, w, y, \
                     stats, N, IH, IW, in_scale, in_shift)
  if (mode == 0) {
    const bool two = conv3_fwd_2wg(), act = in_scale != nullptr;
    if (two && stats && act) XCP_C3F(TH_FWD2, NW_FWD2, true, true);
    else if (two && stats) XCP_C3F(TH_FWD2, NW_FWD2, true, false);
    else if (two && act) XCP_C3F(TH_FWD2, NW_FWD2, false, true);
    else if (two) XCP_C3F(TH_FWD2, NW_FWD2, false, false);
    else if (stats && act) XCP_C3F(TH_FWD, NW_FWD, true, true);
    else if (stats) XCP_C3F(TH_FWD, NW_FWD, true, false);
    else if (act) XCP_C3F(TH_FWD, NW_FWD, false, true);
    else XCP_C3F(TH_FWD, NW_FWD, false, false);
  } else {
    hipLaunchKernelGGL((conv3x3_kernel<64, 32, 2, TH_DGRAD, MAXIW_DGRAD, false, NW_DGRAD, false>), grid, dim3(64 * NW_DGRAD), 0, st,
                       x, w, y, stats, N, IH, IW, nullptr, nullptr);
  }
#undef XCP_C3F
  return (int)hipGetLastError();
}

// slabs (= workgroups) of xcp_conv3x3_wgrad; 0 when the width is unsupported
int xcp_conv3x3_wgrad_parts(int N, int IH, int IW) {
  if (N <= 0 || IH < 3 || IW < 3 || (conv3_wgrad_form() ? IW > WS_APX : IW - 2 > WG_GPX)) return 0;
  int nb, rb;
  wgrad_bands(N, IH - 2, nb, rb);
  return N * nb;
}

// P[parts][64][9 * 32] (fp32 slabs, sum them for dW[co][tap][ci]) = weight gradient of
// Y = conv3x3(X) from dY[N][IH-2][IW-2][64] and X[N][IH][IW][32].  bf16 only.
int xcp_conv3x3_wgrad(const void* dY, const void* X, float* P, int N, int IH, int IW, const float* in_scale,
                      const float* in_shift, hipStream_t st) {
  if (N <= 0) return XCP_OK;
  if (IH < 3 || IW < 3 || (in_scale != nullptr) != (in_shift != nullptr)) return XCP_EINVAL;
  const int form = conv3_wgrad_form();
  if (form ? IW > WS_APX : IW - 2 > WG_GPX) return XCP_EUNSUPPORTED;
  int nb, rb;
  wgrad_bands(N, IH - 2, nb, rb);
  if (form) {
#define XCP_C3W(ACT, CP)                                                                                             \
  hipLaunchKernelGGL((conv3x3_wgrad_s_kernel<ACT, CP>), dim3(N * nb), dim3(512), 0, st, (const bf16*)dY, (const bf16*)X, P, \
                     N, IH, IW, nb, rb, in_scale, in_shift)
    if (in_scale && form == 1) XCP_C3W(true, 1);
    else if (in_scale) XCP_C3W(true, 2);
    else if (form == 1) XCP_C3W(false, 1);
    else XCP_C3W(false, 2);
#undef XCP_C3W
    return (int)hipGetLastError();
  }
  if (in_scale)
    hipLaunchKernelGGL(conv3x3_wgrad_kernel<true>, dim3(N * nb), dim3(512), 0, st, (const bf16*)dY, (const bf16*)X, P, N, IH,
                       IW, nb, rb, in_scale, in_shift);
  else
    hipLaunchKernelGGL(conv3x3_wgrad_kernel<false>, dim3(N * nb), dim3(512), 0, st, (const bf16*)dY, (const bf16*)X, P, N,
                       IH, IW, nb, rb, nullptr, nullptr);
  return (int)hipGetLastError();
}

}  // extern "C"
