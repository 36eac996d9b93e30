// Pointwise 1x1 convolution as an MFMA GEMM (forward, dgrad) and its weight
// gradient (wgrad, split over the pixel dimension).
//
// Reference ops replaced: the pointwise `nn.Conv2d(C, Cout, 1)` of
// SeparableConv2d (Xception.py:42, called at :46), the stride-2 skip conv of
// Block (Xception.py:55, called at :93) and the LSTM input projection
// (x @ W_ih^T for all T at once, XceptionLSTMV.py:18-23 / :67).
//
//   gemm_nt : C[M,N] = A[M,K] . B[N,K]^T       (A = NHWC pixel rows, B = weight
//             [Cout][Cin]); optional row gather of A (stride-s skip conv) and a
//             BatchNorm-statistics epilogue (per-column sum / sum of squares of
//             the stored values, one deterministic partial row per M-tile).
//   gemm_tn : P[s][N,K] = sum_{m in split s} G[m,N]^T X[m,K]   (weight gradient;
//             fp32 partial slabs, reduced deterministically by xcp_colreduce_f32).
//
// Dense bf16 NT calls with enough work run on a 256x256-tile, 8-wave kernel with a
// four-phase quadrant schedule (gemm_nt256k64_kernel); everything else (fp32 parity
// mode, gathered rows, small problems) on a 128x128-tile, 4-wave kernel (each wave
// 64x64 = 4x4 MFMA 16x16 tiles).
// bf16: v_mfma_f32_16x16x32_bf16, fp32: v_mfma_f32_16x16x4_f32 (exact fp32).
// LDS rows are 128 B (one 64-deep bf16 / 32-deep fp32 K-stage), 16-B chunks
// XOR-swizzled with (row>>1)&7 so a 16-lane ds_read_b128 group is conflict-free.
#include "common.h"
#include <stdlib.h>
#include <mutex>
#include <utility>
#include <vector>

namespace {

constexpr int BM = 128, BN = 128, NT = 256;
constexpr int ROWB = 128;                 // bytes per LDS row per K-stage
constexpr int STAGE_BYTES = BM * ROWB;    // one operand, one stage (16 KB)

template <typename T> struct GT;
template <> struct GT<bf16> { static constexpr int EPC = 8; };
template <> struct GT<float> { static constexpr int EPC = 4; };

__device__ __attribute__((aligned(64))) uint4 g_zero16[4];   // zero line for masked LDS-DMA chunks

template <int V> struct IC {
  static constexpr int value = V;
  constexpr operator int() const { return V; }
};
// compile-time loop: f(IC<B>{}), ..., f(IC<E-1>{}) (indices that must fold at instantiation)
template <int B, int E, typename F>
XCP_DEV void static_for(F&& f) {
  if constexpr (B < E) {
    f(IC<B>{});
    static_for<B + 1, E>(f);
  }
}

XCP_DEV int swz(int row, int chunk) { return row * ROWB + ((chunk ^ ((row >> 1) & 7)) << 4); }

// Row gather for the A operand (NT) / X operand (TN):
//   mode 0: row m is at m*ld
//   mode 1: strided 1x1 conv input, m = (n,oh,ow) over OHxOW -> pixel (n, oh*S, ow*S) of HxW
//   mode 2: im2col of a 3x3 stride-1 pad-0 conv, m = (n,oh,ow) over OHxOW, column
//           k = tap*Cg + c -> pixel (n, oh+ky, ow+kx) of HxW, channel c
//   mode 3: transposed im2col (input gradient of that conv), m = (n,h,w) over HxW,
//           k = tap*Cg + c -> pixel (n, h-ky, w-kx) of OHxOW (zero outside), channel c
struct Gather {
  int mode, H, W, OH, OW, S, Cg;
};
struct RowInfo {
  long base;
  int h, w;
  bool ok;
};
template <int GM>
XCP_DEV RowInfo row_info(const Gather& g, int m, int M) {
  RowInfo r{0, 0, 0, m < M};
  if (!r.ok || GM == 0) {
    r.base = r.ok ? m : 0;
    return r;
  }
  if constexpr (GM == 3) {
    const int hw = g.H * g.W, n = m / hw, rem = m - n * hw;
    r.h = rem / g.W;
    r.w = rem - r.h * g.W;
    r.base = (long)n * g.OH * g.OW;
    return r;
  }
  const int ohw = g.OH * g.OW, n = m / ohw, rem = m - n * ohw;
  const int oh = rem / g.OW, ow = rem - oh * g.OW;
  r.base = (long)n * g.H * g.W + (long)oh * g.S * g.W + (long)ow * g.S;
  return r;
}
// element offset of the chunk (row r, column k), or -1 for a zero chunk
template <int GM>
XCP_DEV long chunk_off(const Gather& g, const RowInfo& r, long ld, int k) {
  if constexpr (GM <= 1) return r.base * ld + k;
  const int tap = k / g.Cg, c = k - tap * g.Cg;
  const int ky = tap / 3, kx = tap - ky * 3;
  if constexpr (GM == 2) return (r.base + (long)ky * g.W + kx) * ld + c;
  const int oh = r.h - ky, ow = r.w - kx;
  if (oh < 0 || oh >= g.OH || ow < 0 || ow >= g.OW) return -1;
  return (r.base + (long)oh * g.OW + ow) * ld + c;
}

struct NTArgs {
  const void* A; long lda;
  const void* B; long ldb;
  void* C; long ldc;
  int M, N, K;
  float* stats;           // [gridM][2][N] partial (sum, sumsq) or nullptr
  Gather ga;
  int tqs;                // gemm_nt256p_kernel: tile-queue slot + 1 (0: static tile walk)
  int nsplit;             // gemm_nt256p_kernel: the last nsplit tiles are walked as 2 half tiles each, first
  int khalf;              // gemm_nt256p_kernel: a last K-tile with K % 64 in (0, 32] multiplies its first half only
};

// ---------------------------------------------------------------------------------
// NT kernel: (64*WMW) x 128 output tile per workgroup, WMW x 2 waves, each wave
// 64 x 64 = 4 x 4 MFMA 16x16 tiles.  K advances in 128-byte stages (64 bf16 /
// 32 fp32) through an LDS ring of STAGES slots filled by LDS-DMA (STAGES-1 in
// flight while one is consumed; counted vmcnt + one raw barrier per stage).
// MFMA roles are swapped (weights as the A operand) so each lane ends up holding
// 4 consecutive output columns of one row: the epilogue stages 8-byte pieces and
// takes the BatchNorm statistics from the staged tile while storing it.
constexpr int NBN = 128;

template <int N>
XCP_DEV void wait_vmcnt() {
  if constexpr (N == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  else if constexpr (N == 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
  else if constexpr (N == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  else if constexpr (N == 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  else if constexpr (N == 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else static_assert(N == 0, "unsupported count");
}

template <typename T, int GM, int WMW, int STAGES>
__global__ __launch_bounds__(WMW * 128) void gemm_nt_kernel(NTArgs a) {
  constexpr int NTH = WMW * 128;
  constexpr int BMT = 64 * WMW;
  constexpr int EPC = GT<T>::EPC;
  constexpr int BK = 8 * EPC;
  constexpr int A_BYTES = BMT * ROWB, B_BYTES = NBN * ROWB, SB = A_BYTES + B_BYTES;
  constexpr int A_LOADS = 4, B_LOADS = 8 / WMW, NLOADS = A_LOADS + B_LOADS;
  constexpr int CPITCH = NBN * (int)sizeof(T) + 16;   // epilogue staging row pitch (bytes)
  constexpr int RING = STAGES * SB;
  constexpr int SMEM = RING > BMT * CPITCH ? RING : BMT * CPITCH;
  __shared__ __attribute__((aligned(16))) char smem[SMEM + 2 * (NTH / 64) * NBN * 4];
  float* red = reinterpret_cast<float*>(smem + SMEM);   // [2 (s,q)][waves][NBN]

  const int gridN = (a.N + NBN - 1) / NBN;
  const int gridM = (a.M + BMT - 1) / BMT;
  const int id = xcd_remap(blockIdx.x, gridM * gridN);
  const int bn = id % gridN, bm = id / gridN;
  const int m0 = bm * BMT, n0 = bn * NBN;
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);   // wave-uniform: LDS-DMA destinations (M0) from SGPRs
  const int wm = w >> 1, wn = w & 1;
  const T* A = reinterpret_cast<const T*>(a.A);
  const T* B = reinterpret_cast<const T*>(a.B);

  // LDS-DMA staging (global_load_lds, 16 B per lane, lane-linear 1 KB = 8 rows of
  // 128 B per instruction).  Wave w fills A rows [32w, 32w+32) and B rows
  // [(64/WMW)w, ...).  The XOR chunk swizzle is applied to the per-lane SOURCE
  // address; chunks past K and rows past M / N read a zero line.
  const int pc = lane & 7;
  RowInfo ar[A_LOADS];
  const T* ap[A_LOADS];
  int alc[A_LOADS], blc[B_LOADS];
  const T* bp[B_LOADS];
#pragma unroll
  for (int i = 0; i < A_LOADS; ++i) {
    const int row = w * 32 + i * 8 + (lane >> 3);
    alc[i] = pc ^ ((row >> 1) & 7);
    ar[i] = row_info<GM>(a.ga, m0 + row, a.M);
    ap[i] = ar[i].ok ? A + ar[i].base * a.lda + alc[i] * EPC : nullptr;   // modes 0 / 1
  }
#pragma unroll
  for (int i = 0; i < B_LOADS; ++i) {
    const int row = w * (64 / WMW) + i * 8 + (lane >> 3);
    blc[i] = pc ^ ((row >> 1) & 7);
    const int n = n0 + row;
    bp[i] = n < a.N ? B + (long)n * a.ldb + blc[i] * EPC : nullptr;
  }
  auto glds = [](const void* src, char* dst) {
    __builtin_amdgcn_global_load_lds((const void __attribute__((address_space(1)))*)src,
                                     (void __attribute__((address_space(3)))*)dst, 16, 0, 0);
  };
  auto issue = [&](int kt, int buf) {
    char* sa = smem + buf * SB;
    char* sb = sa + A_BYTES;
    const int kb = kt * BK;
#pragma unroll
    for (int i = 0; i < A_LOADS; ++i) {
      const void* src;
      if constexpr (GM <= 1) {
        src = (ap[i] != nullptr && kb + alc[i] * EPC < a.K) ? (const void*)(ap[i] + kb) : (const void*)g_zero16;
      } else {
        const int k = kb + alc[i] * EPC;
        const long ao = (ar[i].ok && k < a.K) ? chunk_off<GM>(a.ga, ar[i], a.lda, k) : -1;
        src = ao >= 0 ? (const void*)(A + ao) : (const void*)g_zero16;
      }
      glds(src, sa + (w * 32 + i * 8) * ROWB);
    }
#pragma unroll
    for (int i = 0; i < B_LOADS; ++i) {
      const void* src = (bp[i] != nullptr && kb + blc[i] * EPC < a.K) ? (const void*)(bp[i] + kb)
                                                                        : (const void*)g_zero16;
      glds(src, sb + (w * (64 / WMW) + i * 8) * ROWB);
    }
  };

  // acc[mt][nt]: D = W_frag(nt) x A_frag(mt)  ->  lane holds C[m = ..mt*16+fr][n = ..nt*16+4fg+r]
  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = (a.K + BK - 1) / BK;
  constexpr int D = STAGES - 1;
#pragma unroll
  for (int s0 = 0; s0 < D; ++s0)
    if (s0 < nk) issue(s0, s0);
  const int fr = lane & 15, fg = lane >> 4;
  for (int kt = 0; kt < nk; ++kt) {
    // stage kt landed for this wave (later stages may stay in flight), then for all waves
    if constexpr (D >= 2) {
      if (kt + 1 < nk) wait_vmcnt<NLOADS>();
      else wait_vmcnt<0>();
    } else {
      wait_vmcnt<0>();
    }
    __builtin_amdgcn_s_barrier();
    // refill the slot consumed in iteration kt-1 (every wave is past it now)
    if (kt + D < nk) issue(kt + D, (kt + D) % STAGES);
    const char* sa = smem + (kt % STAGES) * SB;
    const char* sb = sa + A_BYTES;
#pragma unroll
    for (int cg = 0; cg < 2; ++cg) {
      const int ch = cg * 4 + fg;
      if constexpr (sizeof(T) == 2) {
        bf16x8 af[4], bfr[4];
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          af[t] = *reinterpret_cast<const bf16x8*>(sa + swz(wm * 64 + t * 16 + fr, ch));
          bfr[t] = *reinterpret_cast<const bf16x8*>(sb + swz(wn * 64 + t * 16 + fr, ch));
        }
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j], af[i], acc[i][j], 0, 0, 0);
      } else {
        f32x4 af[4], bfr[4];
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          af[t] = *reinterpret_cast<const f32x4*>(sa + swz(wm * 64 + t * 16 + fr, ch));
          bfr[t] = *reinterpret_cast<const f32x4*>(sb + swz(wn * 64 + t * 16 + fr, ch));
        }
#pragma unroll
        for (int e = 0; e < 4; ++e)
#pragma unroll
          for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(bfr[j][e], af[i][e], acc[i][j], 0, 0, 0);
      }
    }
  }
  __syncthreads();   // every wave done reading the ring before the epilogue reuses it

  // ---- epilogue: round to T, stage 4-column pieces through LDS
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int row = wm * 64 + i * 16 + fr, col = wn * 64 + j * 16 + fg * 4;
      float v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = acc[i][j][r];
      VecIO<T, 4>::store(reinterpret_cast<T*>(smem + row * CPITCH + col * (int)sizeof(T)), v);
    }
  __syncthreads();
  // ---- coalesced 16-B stores; BN statistics over the stored values
  T* C = reinterpret_cast<T*>(a.C);
  constexpr int CPR = NBN * (int)sizeof(T) / 16;   // 16-B chunks per tile row
  constexpr int RPI = NTH / CPR;                   // rows covered per iteration
  constexpr int ITER = BMT / RPI;
  const int c = tid % CPR, rq = tid / CPR;
  const int n = n0 + c * EPC;
  float s1[EPC], s2[EPC];
#pragma unroll
  for (int e = 0; e < EPC; ++e) s1[e] = s2[e] = 0.f;
#pragma unroll
  for (int i = 0; i < ITER; ++i) {
    const int row = rq + RPI * i;
    const int m = m0 + row;
    const uint4 v = *reinterpret_cast<const uint4*>(smem + row * CPITCH + c * 16);
    if (m < a.M && n < a.N) {
      *reinterpret_cast<uint4*>(C + (long)m * a.ldc + n) = v;
      float f[EPC];
      VecIO<T, EPC>::load(reinterpret_cast<const T*>(&v), f);
#pragma unroll
      for (int e = 0; e < EPC; ++e) {
        s1[e] += f[e];
        s2[e] = fmaf(f[e], f[e], s2[e]);
      }
    }
  }
  if (a.stats) {
    // threads sharing chunk c: tid = c + CPR*rq; fold rq within the wave, then across waves
#pragma unroll
    for (int e = 0; e < EPC; ++e)
#pragma unroll
      for (int o = CPR; o < 64; o <<= 1) {
        s1[e] += __shfl_xor(s1[e], o, 64);
        s2[e] += __shfl_xor(s2[e], o, 64);
      }
    if (lane < CPR) {
#pragma unroll
      for (int e = 0; e < EPC; ++e) {
        red[(0 * (NTH / 64) + w) * NBN + c * EPC + e] = s1[e];
        red[(1 * (NTH / 64) + w) * NBN + c * EPC + e] = s2[e];
      }
    }
    lds_barrier();   // not __syncthreads(): the C stores above must not be waited for
    if (tid < NBN) {
      const int nn = n0 + tid;
      if (nn < a.N) {
        float t1 = 0.f, t2 = 0.f;
#pragma unroll
        for (int q = 0; q < NTH / 64; ++q) {
          t1 += red[(0 * (NTH / 64) + q) * NBN + tid];
          t2 += red[(1 * (NTH / 64) + q) * NBN + tid];
        }
        a.stats[((long)bm * 2 + 0) * a.N + nn] = t1;
        a.stats[((long)bm * 2 + 1) * a.N + nn] = t2;
      }
    }
  }
}

// LDS-free epilogue of the 256x256 NT kernels (acc[i][j][r] = C[m0 + wr*128 + i*16 + fr]
// [n0 + wc*64 + j*16 + fg*4 + r]): lanes fg / fg^1 (16 apart) swap 8-B pieces so each lane
// stores 16 contiguous bytes (one store instruction = 16 rows x 64 B); the BatchNorm partial
// sums of each 128-row half ([ceil(M/128)][2][N]) come from the rounded registers: sums over
// the wave's 8 row fragments, then a 4-step reduce-scatter over the 16 row lanes (30
// shuffles), after which lane fr holds 2 adjacent columns of one statistic.
XCP_DEV void epilogue256_regs(f32x4 (&acc)[8][4], const NTArgs& a, int m0, int n0, int wr, int wc, int fr, int fg) {
  bf16* C = reinterpret_cast<bf16*>(a.C);
  const int bm = m0 / 256, stat_rows = (a.M + 127) / 128;
  const int mrow = m0 + wr * 128 + fr;
  const int ncol = n0 + wc * 64;
  const bool odd = fg & 1;
  float s1[16], s2[16];
#pragma unroll
  for (int q = 0; q < 16; ++q) s1[q] = s2[q] = 0.f;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int m = mrow + i * 16;
    const bool mok = m < a.M;
    uint2 pc[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      pc[j] = make_uint2(pk_bf16(acc[i][j][0], acc[i][j][1]), pk_bf16(acc[i][j][2], acc[i][j][3]));
      const bf16x4 q = __builtin_bit_cast(bf16x4, pc[j]);
      if (mok) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float f = (float)q[r];
          s1[j * 4 + r] += f;
          s2[j * 4 + r] = fmaf(f, f, s2[j * 4 + r]);
        }
      }
    }
    const uint2 snd0 = odd ? pc[0] : pc[1], snd1 = odd ? pc[2] : pc[3];
    uint2 rc0, rc1;
    rc0.x = __shfl_xor(snd0.x, 16, 64);
    rc0.y = __shfl_xor(snd0.y, 16, 64);
    rc1.x = __shfl_xor(snd1.x, 16, 64);
    rc1.y = __shfl_xor(snd1.y, 16, 64);
    const uint4 st0 = odd ? make_uint4(rc0.x, rc0.y, pc[1].x, pc[1].y) : make_uint4(pc[0].x, pc[0].y, rc0.x, rc0.y);
    const uint4 st1 = odd ? make_uint4(rc1.x, rc1.y, pc[3].x, pc[3].y) : make_uint4(pc[2].x, pc[2].y, rc1.x, rc1.y);
    const int c0 = ncol + (odd ? 16 + (fg - 1) * 4 : fg * 4);
    bf16* crow = C + (long)m * a.ldc;
    if (mok && c0 < a.N) *reinterpret_cast<uint4*>(crow + c0) = st0;
    if (mok && c0 + 32 < a.N) *reinterpret_cast<uint4*>(crow + c0 + 32) = st1;
  }
  if (a.stats) {
    // reduce-scatter of v[32] = (s1[16], s2[16]) over the 16 row lanes
    float u[16], v8[8], v4[4], v2[2];
    const bool b3 = fr & 8, b2 = fr & 4, b1 = fr & 2, b0 = fr & 1;
#pragma unroll
    for (int q = 0; q < 16; ++q) u[q] = (b3 ? s2[q] : s1[q]) + __shfl_xor(b3 ? s1[q] : s2[q], 8, 64);
#pragma unroll
    for (int q = 0; q < 8; ++q) v8[q] = (b2 ? u[8 + q] : u[q]) + __shfl_xor(b2 ? u[q] : u[8 + q], 4, 64);
#pragma unroll
    for (int q = 0; q < 4; ++q) v4[q] = (b1 ? v8[4 + q] : v8[q]) + __shfl_xor(b1 ? v8[q] : v8[4 + q], 2, 64);
#pragma unroll
    for (int q = 0; q < 2; ++q) v2[q] = (b0 ? v4[2 + q] : v4[q]) + __shfl_xor(b0 ? v4[q] : v4[2 + q], 1, 64);
    // lane fr holds index 2fr, 2fr+1 of v: statistic fr>>3, j = (fr&7)>>1, r = (fr&1)*2 + q
    const int col = ncol + ((fr & 7) >> 1) * 16 + fg * 4 + (fr & 1) * 2;
    const int srow = bm * 2 + wr;
    if (srow < stat_rows && col < a.N)
      *reinterpret_cast<float2*>(a.stats + ((long)srow * 2 + (fr >> 3)) * a.N + col) = make_float2(v2[0], v2[1]);
  }
}

// ---------------------------------------------------------------------------------
// 256x256 bf16 NT kernel with 64-deep K-tiles (128-B LDS rows, so every 1-KB LDS-DMA
// instruction fetches 8 whole 128-B lines; 64-B rows fetch 16 half lines and measured
// half the load throughput).  Two ring slots of 64 KB.  8 waves (2 M-groups x 4 N),
// wave tile 128x64; a K-tile is four phases, one 64x32 quadrant (16 MFMA) each:
//   Q0 (A-top, B-left)  reads A-top + B-left   issues A-top(t+1)
//   Q1 (A-top, B-right) reads B-right          issues B-left(t+1)
//   Q2 (A-bot, B-right) reads A-bot            issues B-right(t+1)
//   Q3 (A-bot, B-left)  --                     issues A-bot(t+1)
// ("A-top" = the 64 rows of a wave group's first half, both groups: one half-tile of
// 128 rows = 2 LDS-DMA loads per thread).  Tile t+1 goes to the slot of tile t-1,
// whose last reads (Q2 of t-1) retired >= 3 barriers before Q0(t).  Each half-tile is
// retired by a counted vmcnt in the phase BEFORE the one that reads it (so every
// wave has waited before the barrier the reader passes): Q3 retires A-top / B-left of
// t+1, Q0 retires B-right, Q1 retires A-bot.  Wave group 1 runs one barrier behind
// group 0 (its MFMA cluster overlaps group 0's reads and load issue).
constexpr int K_OP = 256 * 128;                // one operand, one slot (32 KB)
// raw buffer resources for LDS-DMA through buffer_load ... lds: SGPR base + one 32-bit VGPR
// offset per lane (cheaper to form and issue than a 64-bit global address).  Lanes only ever
// form in-range offsets or BUF_OOB (>= num_records: the load returns zeros).  num_records is
// the 2 GB maximum rather than the operand's span: measured, the exact span made the NT
// kernel ~10 % slower (tools/gemm_exp.py).  Used while every operand spans < 2 GB
// (xcp_gemm_nt / xcp_gemm_tn check; the 64-bit global-address form otherwise).
constexpr unsigned BUF_OOB = 0x80000000u;
constexpr long BUF_LIMIT = 0x7fffffffL;
constexpr int BUF_RECORDS = 0x7fffffff;
constexpr int BUF_DWORD3 = 0x00020000;   // gfx9 raw buffer descriptor word 3
constexpr int K_SLOT = 2 * K_OP;

XCP_DEV void wait_cnt(int n) {   // outstanding LDS-DMA loads allowed to remain
  if (n >= 4) wait_vmcnt<4>();
  else if (n >= 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
  else wait_vmcnt<0>();
}

template <bool BUF>
__global__ __launch_bounds__(512) void gemm_nt256k64_kernel(NTArgs a) {
  constexpr bool STAG = true;   // wave group 1 runs one barrier behind group 0
  __shared__ __attribute__((aligned(16))) char smem[2 * K_SLOT];
  const int gridN = (a.N + 255) / 256, gridM = (a.M + 255) / 256;
  const int id = xcd_remap(blockIdx.x, gridM * gridN);
  const int bn = id % gridN, bm = id / gridN;
  const int m0 = bm * 256, n0 = bn * 256;
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);   // wave-uniform: LDS-DMA destinations (M0) from SGPRs
  const int wr = w >> 2, wc = w & 3;
  const bf16* A = reinterpret_cast<const bf16*>(a.A);
  const bf16* B = reinterpret_cast<const bf16*>(a.B);

  // half-tile rows loaded by this wave (2 x 8 rows per half-tile):
  //   A-top: (w<4 ? 16w : 128+16(w-4)) + [0,16);  A-bot: that + 64
  //   B-left: 64(w>>1) + 16(w&1) + [0,16);         B-right: that + 32
  const int arow = (w < 4 ? 16 * w : 128 + 16 * (w - 4));
  const int brow = 64 * (w >> 1) + 16 * (w & 1);
  const int lr = lane >> 3;
  const bf16* src[4][2];   // [half-tile][i]
  unsigned voff[4][2];     // BUF: byte offsets into the A / B buffer resources (OOB -> zeros)
  int kc8[4][2];
#pragma unroll
  for (int h = 0; h < 4; ++h)
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const bool isA = (h == 0 || h == 3);
      const int row = (isA ? arow + (h == 3 ? 64 : 0) : brow + (h == 2 ? 32 : 0)) + i * 8 + lr;
      kc8[h][i] = ((lane & 7) ^ ((row >> 1) & 7)) * 8;
      src[h][i] = isA ? A + (long)min(m0 + row, a.M - 1) * a.lda + kc8[h][i]
                      : B + (long)min(n0 + row, a.N - 1) * a.ldb + kc8[h][i];
      const bool ok = isA ? m0 + row < a.M : n0 + row < a.N;
      voff[h][i] = ok ? (unsigned)(isA ? ((long)(m0 + row) * a.lda + kc8[h][i]) * 2
                                       : ((long)(n0 + row) * a.ldb + kc8[h][i]) * 2)
                      : BUF_OOB;
    }
  const void* zero = g_zero16;
  asm volatile("" : "+v"(zero));
  const __amdgpu_buffer_rsrc_t rA = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(a.A), (short)0, BUF_RECORDS,
                                                                       BUF_DWORD3);
  const __amdgpu_buffer_rsrc_t rB = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(a.B), (short)0, BUF_RECORDS,
                                                                       BUF_DWORD3);
  auto glds = [](const void* p, char* dst) {
    __builtin_amdgcn_global_load_lds((const void __attribute__((address_space(1)))*)p,
                                     (void __attribute__((address_space(3)))*)dst, 16, 0, 0);
  };
  // half-tile h of K-tile kt: h 0 = A-top, 1 = B-left, 2 = B-right, 3 = A-bot
  auto issue = [&](int h, int kt) {
    const bool isA = (h == 0 || h == 3);
    const int row0 = isA ? arow + (h == 3 ? 64 : 0) : brow + (h == 2 ? 32 : 0);
    char* d = smem + (kt & 1) * K_SLOT + (isA ? 0 : K_OP) + row0 * 128;
    const int kb = kt * 64;
    if constexpr (BUF) {
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const unsigned o = kb + kc8[h][i] < a.K ? voff[h][i] + kb * 2 : BUF_OOB;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(isA ? rA : rB, (__attribute__((address_space(3))) void*)(d + i * 1024),
                                                 16, o, 0, 0, 0);
      }
    } else if (kb + 64 <= a.K) {
#pragma unroll
      for (int i = 0; i < 2; ++i) glds(src[h][i] + kb, d + i * 1024);
    } else {
#pragma unroll
      for (int i = 0; i < 2; ++i) glds(kb + kc8[h][i] < a.K ? (const void*)(src[h][i] + kb) : zero, d + i * 1024);
    }
  };

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = (a.K + 63) / 64;
#pragma unroll
  for (int h = 0; h < 4; ++h) issue(h, 0);
  wait_vmcnt<0>();
  __builtin_amdgcn_s_barrier();
  if (STAG && wr == 1) __builtin_amdgcn_s_barrier();

  const int fr = lane & 15, fg = lane >> 4;
  bf16x8 af[4][2], bl[2][2], br[2][2];   // [frag][k-step]
  auto mfma_q = [&](int ih, const bf16x8 (&b)[2][2], int jh) {
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[ih * 4 + i][jh * 2 + j] =
              __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[j][ks], af[i][ks], acc[ih * 4 + i][jh * 2 + j], 0, 0, 0);
  };
  auto sync_mfma = [&](int ih, const bf16x8 (&b)[2][2], int jh) {
    __builtin_amdgcn_s_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
    mfma_q(ih, b, jh);
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_s_barrier();
  };
  for (int kt = 0; kt < nk; ++kt) {
    const char* sa = smem + (kt & 1) * K_SLOT;
    const char* sb = sa + K_OP;
    const bool nxt = kt + 1 < nk;
    // Q0: A-top x B-left
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
#pragma unroll
      for (int j = 0; j < 2; ++j)
        bl[j][ks] = *reinterpret_cast<const bf16x8*>(sb + swz(wc * 64 + j * 16 + fr, ks * 4 + fg));
#pragma unroll
      for (int i = 0; i < 4; ++i)
        af[i][ks] = *reinterpret_cast<const bf16x8*>(sa + swz(wr * 128 + i * 16 + fr, ks * 4 + fg));
    }
    if (nxt) issue(0, kt + 1);
    wait_cnt(2 + (nxt ? 2 : 0));          // B-right(kt) for Q1
    sync_mfma(0, bl, 0);
    // Q1: A-top x B-right
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int j = 0; j < 2; ++j)
        br[j][ks] = *reinterpret_cast<const bf16x8*>(sb + swz(wc * 64 + 32 + j * 16 + fr, ks * 4 + fg));
    if (nxt) issue(1, kt + 1);
    wait_cnt(nxt ? 4 : 0);                // A-bot(kt) for Q2
    sync_mfma(0, br, 1);
    // Q2: A-bot x B-right
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < 4; ++i)
        af[i][ks] = *reinterpret_cast<const bf16x8*>(sa + swz(wr * 128 + 64 + i * 16 + fr, ks * 4 + fg));
    if (nxt) issue(2, kt + 1);
    sync_mfma(1, br, 1);
    // Q3: A-bot x B-left
    if (nxt) {
      issue(3, kt + 1);
      wait_cnt(4);                        // A-top / B-left(kt+1) for Q0(kt+1)
    }
    sync_mfma(1, bl, 0);
  }
  if (STAG && wr == 0) __builtin_amdgcn_s_barrier();
  epilogue256_regs(acc, a, m0, n0, wr, wc, fr, fg);
}

// ---------------------------------------------------------------------------------
// Persistent 256x256 NT kernel: the main loop of gemm_nt256k64_kernel, one workgroup per CU
// walking its tiles (round r: tile r * grid + its XCD-remapped slot, so each round keeps the
// A-row sharing of the one-shot kernel).  Per tile the one-shot kernel pays a fixed cost of
// ~8-15 us at K = 736 (tools/gemm_probe.py: launch boundary, the first K-tile's fill latency and
// the epilogue's 128 KB of stores, all CUs storing at once) against ~1.55 us per 64-deep
// K-tile.  Here the next tile's first K-tile is issued BEFORE this tile's epilogue, so its fill
// runs under the epilogue's conversion and store issue, and the stores drain under the next
// tile's first K-tile: the counted waits of that K-tile allow the S epilogue stores (issued
// after the prefetch, before the K-tile-1 loads) to stay in flight; the first wait that needs
// a K-tile-1 load (phase Q3) retires them.  Every epilogue store is a buffer store whose masked
// lanes get an out-of-range offset, so each wave issues exactly S store instructions and the
// counts are exact (a skipped, fully masked store would make a count one short: a race).
XCP_DEV void vm_wait(int n) {   // s_waitcnt vmcnt(n), n in [0, 63] (folds when n is constant)
  switch (n < 0 ? 0 : n > 63 ? 63 : n) {
#define XCP_VMW(k) case k: asm volatile("s_waitcnt vmcnt(" #k ")" ::: "memory"); break;
    XCP_VMW(0) XCP_VMW(1) XCP_VMW(2) XCP_VMW(3) XCP_VMW(4) XCP_VMW(5) XCP_VMW(6) XCP_VMW(7)
    XCP_VMW(8) XCP_VMW(9) XCP_VMW(10) XCP_VMW(11) XCP_VMW(12) XCP_VMW(13) XCP_VMW(14) XCP_VMW(15)
    XCP_VMW(16) XCP_VMW(17) XCP_VMW(18) XCP_VMW(19) XCP_VMW(20) XCP_VMW(21) XCP_VMW(22) XCP_VMW(23)
    XCP_VMW(24) XCP_VMW(25) XCP_VMW(26) XCP_VMW(27) XCP_VMW(28) XCP_VMW(29) XCP_VMW(30) XCP_VMW(31)
    XCP_VMW(32) XCP_VMW(33) XCP_VMW(34) XCP_VMW(35) XCP_VMW(36) XCP_VMW(37) XCP_VMW(38) XCP_VMW(39)
    XCP_VMW(40) XCP_VMW(41) XCP_VMW(42) XCP_VMW(43) XCP_VMW(44) XCP_VMW(45) XCP_VMW(46) XCP_VMW(47)
    XCP_VMW(48) XCP_VMW(49) XCP_VMW(50) XCP_VMW(51) XCP_VMW(52) XCP_VMW(53) XCP_VMW(54) XCP_VMW(55)
    XCP_VMW(56) XCP_VMW(57) XCP_VMW(58) XCP_VMW(59) XCP_VMW(60) XCP_VMW(61) XCP_VMW(62) XCP_VMW(63)
#undef XCP_VMW
  }
}

typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef int i32x2 __attribute__((ext_vector_type(2)));

// epilogue256_regs with buffer stores (always issued; OOB offset for masked lanes):
// 16 C stores per lane, + 1 statistics store when STATS
// (FENCE: no instruction moves across a row block's end -- for accumulators in AGPRs, whose reads the
// scheduler otherwise hoists all at once into VGPRs.  SKIP: a store whose every lane is out of range is not
// issued (wave-uniform test), and the count of store instructions issued is returned: a store dropped whole by
// the range check was seen to retire its vmcnt ahead of older loads, which a counted wait cannot allow for)
template <bool STATS, typename Get, bool FENCE = false, bool SKIP = false>
XCP_DEV int epilogue256_get(Get acc, const NTArgs& a, __amdgpu_buffer_rsrc_t rC, __amdgpu_buffer_rsrc_t rS, int m0,
                            int n0, int wr, int wc, int fr, int fg, int side = 0) {
  int issued = 0;
  const int bm = m0 / 256, stat_rows = (a.M + 127) / 128;
  const int mrow = m0 + wr * 128 + fr;
  const int ncol = n0 + wc * 64;
  const bool odd = fg & 1;
  float s1[16], s2[16];
#pragma unroll
  for (int q = 0; q < 16; ++q) s1[q] = s2[q] = 0.f;
  const int c0 = ncol + (odd ? 16 + (fg - 1) * 4 : fg * 4);
  static_for<0, 8>([&](auto i) {
    const int m = mrow + i * 16;
    const bool mok = m < a.M;
    uint2 pc[4];
    static_for<0, 4>([&](auto j) {
      pc[j] = make_uint2(pk_bf16(acc(i, j, 0), acc(i, j, 1)), pk_bf16(acc(i, j, 2), acc(i, j, 3)));
      const bf16x4 q = __builtin_bit_cast(bf16x4, pc[j]);
      if constexpr (STATS) {   // (branch-free: rows past M add zero)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float f = mok ? (float)q[r] : 0.f;
          s1[j * 4 + r] += f;
          s2[j * 4 + r] = fmaf(f, f, s2[j * 4 + r]);
        }
      }
    });
    const uint2 snd0 = odd ? pc[0] : pc[1], snd1 = odd ? pc[2] : pc[3];
    uint2 rc0, rc1;
    rc0.x = __shfl_xor(snd0.x, 16, 64);
    rc0.y = __shfl_xor(snd0.y, 16, 64);
    rc1.x = __shfl_xor(snd1.x, 16, 64);
    rc1.y = __shfl_xor(snd1.y, 16, 64);
    const uint4 st0 = odd ? make_uint4(rc0.x, rc0.y, pc[1].x, pc[1].y) : make_uint4(pc[0].x, pc[0].y, rc0.x, rc0.y);
    const uint4 st1 = odd ? make_uint4(rc1.x, rc1.y, pc[3].x, pc[3].y) : make_uint4(pc[2].x, pc[2].y, rc1.x, rc1.y);
    const unsigned rowb = (unsigned)((long)m * a.ldc * 2);
    // (a half tile stores only its side: st0 holds the left 32 columns of the wave, st1 the right 32)
    const unsigned o0 = (mok && c0 < a.N && side != 2) ? rowb + (unsigned)c0 * 2 : BUF_OOB;
    const unsigned o1 = (mok && c0 + 32 < a.N && side != 1) ? rowb + (unsigned)(c0 + 32) * 2 : BUF_OOB;
    // non-temporal (nt) C stores: the tile's 128 KB leave as streaming writes, so the round's 32 MB burst does
    // not sit in the L2s as ordinary dirty lines ahead of the next kernel's reads (the depthwise forward that
    // reads this output ran 0.433 -> 0.48 of HBM in the step, the op itself 130 -> 125 us, the step +0.9 %;
    // sc1 write-through measured slower: profiles/r06_nt_cstore_ab.txt)
    // (A/B: tools/exp/gemm_cnt.hip / gemm_csc1.hip were this file with the policy argument 2 / 16 instead of 0;
    // a runtime-selected policy costs the persistent kernel 18 more spilled SGPRs, so it is fixed here)
    if constexpr (SKIP) {
      const bool rows = m0 + wr * 128 + i * 16 < a.M;   // (wave-uniform: some row of the block in range)
      if (rows && ncol < a.N) {
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(i32x4, st0), rC, (int)o0, 0, 2);
        ++issued;
      }
      if (rows && ncol + 32 < a.N) {
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(i32x4, st1), rC, (int)o1, 0, 2);
        ++issued;
      }
    } else {
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(i32x4, st0), rC, (int)o0, 0, 2);
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(i32x4, st1), rC, (int)o1, 0, 2);
    }
    if constexpr (FENCE) __builtin_amdgcn_sched_barrier(0);
  });
  if constexpr (STATS) {
    float u[16], v8[8], v4[4], v2[2];
    const bool b3 = fr & 8, b2 = fr & 4, b1 = fr & 2, b0 = fr & 1;
#pragma unroll
    for (int q = 0; q < 16; ++q) u[q] = (b3 ? s2[q] : s1[q]) + __shfl_xor(b3 ? s1[q] : s2[q], 8, 64);
#pragma unroll
    for (int q = 0; q < 8; ++q) v8[q] = (b2 ? u[8 + q] : u[q]) + __shfl_xor(b2 ? u[q] : u[8 + q], 4, 64);
#pragma unroll
    for (int q = 0; q < 4; ++q) v4[q] = (b1 ? v8[4 + q] : v8[q]) + __shfl_xor(b1 ? v8[q] : v8[4 + q], 2, 64);
#pragma unroll
    for (int q = 0; q < 2; ++q) v2[q] = (b0 ? v4[2 + q] : v4[q]) + __shfl_xor(b0 ? v4[q] : v4[2 + q], 1, 64);
    const int col = ncol + ((fr & 7) >> 1) * 16 + fg * 4 + (fr & 1) * 2;
    const int srow = bm * 2 + wr;
    const bool sok = side == 0 || (side == 1) == (((fr & 7) >> 1) < 2);   // (a half tile: its side's columns)
    const unsigned so = (srow < stat_rows && col < a.N && sok)
                            ? (unsigned)((((long)srow * 2 + (fr >> 3)) * a.N + col) * 4) : BUF_OOB;
    if (!SKIP || (bm * 2 + wr < stat_rows && ncol < a.N)) {
      __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(i32x2, make_float2(v2[0], v2[1])), rS, (int)so, 0, 0);
      ++issued;
    }
  }
  return issued;
}

template <bool STATS>
XCP_DEV void epilogue256_buf(f32x4 (&acc)[8][4], const NTArgs& a, __amdgpu_buffer_rsrc_t rC,
                             __amdgpu_buffer_rsrc_t rS, int m0, int n0, int wr, int wc, int fr, int fg, int side = 0) {
  epilogue256_get<STATS>([&](int i, int j, int r) { return acc[i][j][r]; }, a, rC, rS, m0, n0, wr, wc, fr, fg, side);
}

// Tile counters of the persistent NT kernel, one per (device, stream) slot: a workgroup takes its first
// tile by its slot and every further one from the counter (fetched by one thread at a tile's start,
// consumed after the K loop), so the workgroups that run absorb the tiles of those that start late
// (CUs held by the side stream's weight-gradient GEMM).  Each launch fetches exactly `tiles` times
// (one failing fetch per active workgroup ends its walk), so the fetch that returns tiles - 1 is the
// last and resets the counter for the next launch (graph replays included).
__device__ int g_nt_tq[64];

// PF2 (opt-in, XCP_NT_PF2=1; C bitwise equal, but the step measured 0.4-0.6 % slower and the in-step
// middle-flow op 754 -> 738 TFLOP/s, the K = 128 entry shapes up to 11 % slower alone:
// profiles/r06_nt_pf2_ab.txt): at a tile boundary the next tile's first TWO K-tiles (both ring slots) are issued ahead of this tile's
// epilogue stores, so the stores stay in flight through the next tile's K-tile 0 and most of K-tile 1 (the
// first wait that retires them is K-tile 1's phase Q3) instead of K-tile 0's Q3: the round's 32 MB store
// burst gets two K-tiles to drain instead of one.  (The first tile has no stores ahead of it: its waits
// count without them.  Dropped out-of-range stores in their place measured wrong C: their counts may retire
// ahead of older loads.)
template <bool STATS, bool HALF, bool PF2>
__global__ __launch_bounds__(512) void gemm_nt256p_kernel(NTArgs a) {
  constexpr int S_ST = 16 + (STATS ? 1 : 0);   // store instructions per wave per epilogue
  // (+ 16 B for the tile-queue broadcast: in the ring's LDS object, since a second object would give the
  // LDS accesses alias scopes and hipcc would drain the DMA ahead of the fragment reads)
  __shared__ __attribute__((aligned(16))) char smem[2 * K_SLOT + 16];
  int* const s_next = reinterpret_cast<int*>(smem + 2 * K_SLOT);
  int* const tq = a.tqs > 0 ? g_nt_tq + (a.tqs - 1) : nullptr;
  const int gridN = (a.N + 255) / 256, gridM = (a.M + 255) / 256;
  const int tiles = gridM * gridN, nwg = gridDim.x;
  // work items: the last nsplit tiles as 2 half tiles each (side 1: the B-left 32 columns of every wave's 64,
  // side 2: the B-right 32), walked FIRST, then the other tiles whole (side 0).  A half tile runs only its
  // side's two quadrant phases, so the workgroups that start with one reach their tile boundaries (and their
  // epilogue stores) about half a tile out of step with the rest: the rounds' store bursts no longer coincide.
  const int nsplit = HALF ? a.nsplit : 0, nhalf = 2 * nsplit, items = tiles + nsplit;
  auto item_tile = [&](int it, int& side) {
    if constexpr (HALF) {
      if (it < nhalf) {
        side = 1 + (it & 1);
        return tiles - nsplit + (it >> 1);
      }
    }
    side = 0;
    return it - nhalf;
  };
  const int slot = xcd_remap(blockIdx.x, nwg);
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);   // wave-uniform: LDS-DMA destinations (M0) from SGPRs
  const int wr = w >> 2, wc = w & 3;
  const int arow = (w < 4 ? 16 * w : 128 + 16 * (w - 4));
  const int brow = 64 * (w >> 1) + 16 * (w & 1);
  const int lr = lane >> 3;
  int rowt[4][2], kc8[4][2];
#pragma unroll
  for (int h = 0; h < 4; ++h)
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const bool isA = (h == 0 || h == 3);
      rowt[h][i] = (isA ? arow + (h == 3 ? 64 : 0) : brow + (h == 2 ? 32 : 0)) + i * 8 + lr;
      kc8[h][i] = ((lane & 7) ^ ((rowt[h][i] >> 1) & 7)) * 8;
    }
  const __amdgpu_buffer_rsrc_t rA = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(a.A), (short)0, BUF_RECORDS,
                                                                       BUF_DWORD3);
  const __amdgpu_buffer_rsrc_t rB = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(a.B), (short)0, BUF_RECORDS,
                                                                       BUF_DWORD3);
  const __amdgpu_buffer_rsrc_t rC = __builtin_amdgcn_make_buffer_rsrc(a.C, (short)0, BUF_RECORDS, BUF_DWORD3);
  const __amdgpu_buffer_rsrc_t rS = __builtin_amdgcn_make_buffer_rsrc(STATS ? (void*)a.stats : a.C, (short)0,
                                                                       BUF_RECORDS, BUF_DWORD3);
  unsigned voff[4][2];
  auto set_tile = [&](int m0, int n0, int side) {
#pragma unroll
    for (int h = 0; h < 4; ++h)
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const bool isA = (h == 0 || h == 3);
        const int r = (isA ? m0 : n0) + rowt[h][i];
        // (a half tile's other B half is not fetched: its DMA slots load the zero line)
        const bool ok = (isA ? r < a.M : r < a.N) && !(HALF && ((h == 1 && side == 2) || (h == 2 && side == 1)));
        voff[h][i] = ok ? (unsigned)(((long)r * (isA ? a.lda : a.ldb) + kc8[h][i]) * 2) : BUF_OOB;
      }
  };
  auto issue = [&](int h, int kt) {
    const bool isA = (h == 0 || h == 3);
    const int row0 = isA ? arow + (h == 3 ? 64 : 0) : brow + (h == 2 ? 32 : 0);
    char* d = smem + (kt & 1) * K_SLOT + (isA ? 0 : K_OP) + row0 * 128;
    const int kb = kt * 64;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const unsigned o = kb + kc8[h][i] < a.K ? voff[h][i] + kb * 2 : BUF_OOB;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(isA ? rA : rB, (__attribute__((address_space(3))) void*)(d + i * 1024),
                                               16, o, 0, 0, 0);
    }
  };

  f32x4 acc[8][4];
  const int nk = (a.K + 63) / 64;
  // (XCP_NT_KHALF=0: every K-tile whole; the A/B switch, read per launch on the host)
  const bool khalf = a.khalf && (a.K & 63) != 0 && (a.K & 63) <= 32;
  const int fr = lane & 15, fg = lane >> 4;
  bf16x8 af[4][2], bl[2][2], br[2][2];
  // NKS: 32-deep halves of the K-tile to multiply (1: the last K-tile of a K with K % 64 in (0, 32], whose
  // second half is all zero lines -- adding its +0 products leaves every accumulator's bits unchanged)
  bool lastk = false;   // (wave-uniform) the K-tile being multiplied is the last one
  auto mfma_q = [&](int ih, const bf16x8 (&b)[2][2], int jh, auto nks) {
    constexpr int NKS = decltype(nks)::value;
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) {
      if (ks == 1 && khalf && lastk) break;
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[ih * 4 + i][jh * 2 + j] =
              __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[j][ks], af[i][ks], acc[ih * 4 + i][jh * 2 + j], 0, 0, 0);
    }
  };
  int side = 0;   // of the current item (wave-uniform)
  auto sync_mfma = [&](int ih, const bf16x8 (&b)[2][2], int jh, auto nks) {
    __builtin_amdgcn_s_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    if (!HALF || side != 2 - jh) {   // (a half tile skips the other side's quadrants)
      __builtin_amdgcn_s_setprio(1);
      mfma_q(ih, b, jh, nks);
      __builtin_amdgcn_s_setprio(0);
    }
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
  };

  int t = slot;
  if (t >= items) return;
  int tile = item_tile(t, side);
  int m0 = (tile / gridN) * 256, n0 = (tile % gridN) * 256;
  set_tile(m0, n0, side);
#pragma unroll
  for (int h = 0; h < 4; ++h) issue(h, 0);
  if constexpr (PF2) {
    if (nk > 1)
#pragma unroll
      for (int h = 0; h < 4; ++h) issue(h, 1);
  }
  int extra = 0;   // epilogue stores of the previous tile still allowed in flight during K-tile 0
  while (true) {
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    if constexpr (PF2) {   // K-tile 0 landed (K-tile 1's loads and the previous epilogue's stores may remain)
      if (nk > 1) {
        if (extra) vm_wait(8 + S_ST);
        else vm_wait(8);
      } else if (extra) vm_wait(S_ST);
      else wait_vmcnt<0>();
    } else if (extra) vm_wait(S_ST);   // K-tile 0 landed (the previous epilogue's stores may still drain)
    else wait_vmcnt<0>();
    // (thread 0) the queue position of the next tile, by inline asm: the compiler would wait for the
    // returned value at once (vmcnt(0), draining the prefetch).  Issued after the wait above and before
    // K-tile 1's loads, it has retired by the time the K loop waits for those (VMEM returns in order).
    unsigned nxt = 0;
    if (tq && tid == 0)
      asm volatile("global_atomic_add %0, %1, %2, off sc0" : "=v"(nxt) : "v"(tq), "v"(1u) : "memory");
    __builtin_amdgcn_s_barrier();
    if (wr == 1) __builtin_amdgcn_s_barrier();
    // one 64-deep K-tile.  MODE 1 (kt == 0): its data was retired by the wait above, so the two
    // in-tile waits are skipped (they would otherwise also wait for the previous epilogue's stores);
    // with PF2 it issues nothing (K-tile 1 is in flight) and its Q3 wait leaves the stores in flight.
    // MODE 2 (PF2, kt == 1): the previous epilogue's S_ST stores sit between K-tile 1's loads and K-tile
    // 2's, so its Q0 / Q1 waits allow S_ST more; its Q3 wait retires them.
    auto ktile = [&](int kt, auto mode, auto nks) {
      constexpr int MODE = decltype(mode)::value;
      constexpr bool ISSUE = !(PF2 && MODE == 1);
      const char* sa = smem + (kt & 1) * K_SLOT;
      const char* sb = sa + K_OP;
      const bool nxt = kt + 1 < nk;
      lastk = !nxt;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
#pragma unroll
        for (int j = 0; j < 2; ++j)
          bl[j][ks] = *reinterpret_cast<const bf16x8*>(sb + swz(wc * 64 + j * 16 + fr, ks * 4 + fg));
#pragma unroll
        for (int i = 0; i < 4; ++i)
          af[i][ks] = *reinterpret_cast<const bf16x8*>(sa + swz(wr * 128 + i * 16 + fr, ks * 4 + fg));
      }
      if (ISSUE && nxt) issue(0, kt + 1);
      if constexpr (MODE == 0) wait_cnt(2 + (nxt ? 2 : 0));   // B-right(kt) for Q1
      if constexpr (MODE == 2) {
        if (nxt) {
          if (extra) vm_wait(4 + S_ST);
          else vm_wait(4);
        } else if (extra) vm_wait(2 + S_ST);
        else vm_wait(2);
      }
      sync_mfma(0, bl, 0, nks);
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          br[j][ks] = *reinterpret_cast<const bf16x8*>(sb + swz(wc * 64 + 32 + j * 16 + fr, ks * 4 + fg));
      if (ISSUE && nxt) issue(1, kt + 1);
      if constexpr (MODE == 0) wait_cnt(nxt ? 4 : 0);         // A-bot(kt) for Q2
      if constexpr (MODE == 2) {   // (nk == 2: everything, the tile-queue fetch included, is retired here)
        if (!nxt) wait_vmcnt<0>();
        else if (extra) vm_wait(4 + S_ST);
        else vm_wait(4);
      }
      sync_mfma(0, br, 1, nks);
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int i = 0; i < 4; ++i)
          af[i][ks] = *reinterpret_cast<const bf16x8*>(sa + swz(wr * 128 + 64 + i * 16 + fr, ks * 4 + fg));
      if (ISSUE && nxt) issue(2, kt + 1);
      sync_mfma(1, br, 1, nks);
      if (nxt) {
        if constexpr (ISSUE) {
          issue(3, kt + 1);
          wait_cnt(4);   // A-top / B-left(kt+1) for Q0(kt+1); also retires the previous epilogue's stores
        } else if (extra) {
          vm_wait(4 + S_ST);   // A-top / B-left(1): B-right / A-bot(1) and the stores may remain
        } else {
          vm_wait(4);
        }
      }
      sync_mfma(1, bl, 0, nks);
    };
    if constexpr (PF2) {
      ktile(0, IC<1>{}, IC<2>{});
      if (nk > 1) ktile(1, IC<2>{}, IC<2>{});
      for (int kt = 2; kt < nk; ++kt) ktile(kt, IC<0>{}, IC<2>{});
    } else {
      ktile(0, IC<1>{}, IC<2>{});
      for (int kt = 1; kt < nk; ++kt) ktile(kt, IC<0>{}, IC<2>{});
    }
    if (wr == 0) __builtin_amdgcn_s_barrier();   // every wave is done reading both ring slots
    const int cm0 = m0, cn0 = n0, cside = side;
    if (tq) {
      if (tid == 0) {
        asm volatile("" : "+v"(nxt));   // (used only here, after the K loop's waits)
        *s_next = (int)nxt;
        if ((int)nxt == items - 1) __hip_atomic_store(tq, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      lds_barrier();
      t = nwg + __builtin_amdgcn_readfirstlane(*s_next);
    } else {
      t += nwg;
    }
    const bool more = t < items;
    if (more) {   // the next tile's first K-tile, ahead of this tile's stores
      tile = item_tile(t, side);
      m0 = (tile / gridN) * 256;
      n0 = (tile % gridN) * 256;
      set_tile(m0, n0, side);
#pragma unroll
      for (int h = 0; h < 4; ++h) issue(h, 0);
      if constexpr (PF2) {
        if (nk > 1)
#pragma unroll
          for (int h = 0; h < 4; ++h) issue(h, 1);
      }
    }
    epilogue256_buf<STATS>(acc, a, rC, rS, cm0, cn0, wr, wc, fr, fg, HALF ? cside : 0);
    if (!more) break;
    extra = S_ST;
  }
}

// ---------------------------------------------------------------------------------
// Persistent 256x256 NT kernel at ONE wave per SIMD (gemm_nt4w_kernel; opt-in XCP_NT_4W=1 while measured).
//
// The 8-wave kernels above split a 256x256 tile into 128x64 wave tiles (two waves per SIMD) and pay
// 8 s_barrier per 64-deep K-tile around 16-MFMA phases (profiles/r04_nt_probe.txt: that skeleton is
// 0.45 us per K-tile over 0.86 us of MFMA issue).  Here 4 waves each own a 128x128 quarter (64
// accumulators, 256 registers; 512 per wave at one wave per SIMD):
//   * K advances in 32-deep steps through a 4-slot LDS ring (32 KB per step: A and B 256 rows x 64 B);
//     steps g+1 .. g+3 are in flight while step g computes, and step g+4 is issued into g's slot;
//   * ONE barrier per step: after it every wave's pieces of step g+1 have landed (each wave waits for
//     its own by a counted vmcnt) and every wave has its step-g fragments in registers (lgkmcnt(0)
//     before the barrier), so g's slot is refilled and g+1's fragments are read while g's 64 MFMAs
//     run (fragments double-buffered in registers);
//   * the fill is one continuous stream over the workgroup's tiles: a tile's last steps issue the next
//     tile's first ones, so there is no per-tile prologue; the epilogue's stores (32 + 1 per wave) then
//     stay in flight through the next tile's first three steps.  Past the walk's end the stream
//     re-issues its last tile's first step (real loads), so every step counts the same instructions.
// Operand images: rows of 64 B, 16-B chunk c of row r at chunk c ^ f((r >> 2) & 3), f = (0, 2, 3, 1):
// every lane group of a ds_read_b128 fragment read (rows fr, chunks fg) then covers 16 distinct bank
// quads.  LDS-DMA writes 16 B per lane at consecutive addresses, so the swizzle is applied to the
// source: lane l of a piece fetches row (l >> 2), logical chunk (l & 3) ^ f(l >> 4).
// C and the BN statistics: the 256p kernel's operand order, K order, epilogue packing and statistics
// reduction tree, so both are bitwise equal to it.
constexpr int W4_OP = 256 * 64;     // one operand of one 32-deep K-step (16 KB)
constexpr int W4_SLOT = 2 * W4_OP;  // A + B
constexpr int W4_NS = 4;

XCP_DEV int w4_f(int q) { return (0x1320 >> (q * 4)) & 3; }
// the MFMA by inline asm with the accumulator pinned to AGPRs and the operands to VGPRs: with 256 accumulator
// registers and 128 fragment registers the builtin's register-class choice shuttled accumulators between the
// two files (v_accvgpr_write / read around every MFMA, and spills).  hipcc pads no hazard for an asm MFMA:
// the accumulators are zeroed >= 4 wait states before the first one reads them and read back only after an
// s_nop pad (w4_pad), and the fragments come from ds_read (no VALU-write -> MFMA-read hazard)
XCP_DEV void w4_mfma(f32x4& c, const bf16x8& a, const bf16x8& b) {
  asm("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(c) : "v"(a), "v"(b));
}
XCP_DEV void w4_pad() { asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory"); }
XCP_DEV int w4_swz(int r, int c) { return r * 64 + ((c ^ w4_f((r >> 2) & 3)) << 4); }

template <bool STATS, bool W4_ILV>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1))) void gemm_nt4w_kernel(NTArgs a) {
  constexpr bool w4_ilv = W4_ILV;
  // the ring, then 16 KB of zeros: the fragments of a padding step are read from there
  __shared__ __attribute__((aligned(16))) char smem[W4_NS * W4_SLOT + W4_OP];
  const int gridN = (a.N + 255) / 256, gridM = (a.M + 255) / 256;
  const int tiles = gridM * gridN, nwg = gridDim.x;
  const int slot = xcd_remap(blockIdx.x, nwg);
  if (slot >= tiles) return;
  for (int i = threadIdx.x; i < W4_OP / 16; i += 256)
    reinterpret_cast<uint4*>(smem + W4_NS * W4_SLOT)[i] = make_uint4(0u, 0u, 0u, 0u);
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = w >> 1, wc = w & 1;
  const int fr = lane & 15, fg = lane >> 4;
  // 32-deep steps: nkr of them, walked as an even number nk (an odd count gets one more step that loads step 0's
  // data again -- no load past K is ever issued whole -- and multiplies fragments read from the zero block:
  // the accumulators start at +0, so adding the +-0 products leaves every bit as it was)
  const int nkr = (a.K + 31) / 32, nk = (nkr + 1) & ~1;
  const __amdgpu_buffer_rsrc_t rA = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(a.A), (short)0, BUF_RECORDS,
                                                                       BUF_DWORD3);
  const __amdgpu_buffer_rsrc_t rB = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(a.B), (short)0, BUF_RECORDS,
                                                                       BUF_DWORD3);
  const __amdgpu_buffer_rsrc_t rC = __builtin_amdgcn_make_buffer_rsrc(a.C, (short)0, BUF_RECORDS, BUF_DWORD3);
  const __amdgpu_buffer_rsrc_t rS = __builtin_amdgcn_make_buffer_rsrc(STATS ? (void*)a.stats : a.C, (short)0,
                                                                       BUF_RECORDS, BUF_DWORD3);
  // ---- the fill stream: wave w loads rows w*64 .. w*64+63 of both operands, 4 pieces of 16 rows each
  const int lrow = w * 64 + (lane >> 2);           // + 16 i
  const int lc = (lane & 3) ^ w4_f(lane >> 4);    // logical chunk of this lane ((row >> 2) & 3 == lane >> 4)
  unsigned va[4], vb[4];                          // this lane's chunk offsets in the fill tile (BUF_OOB: past M / N)
  int dt = slot, dks = 0, nfill = 0;              // fill pointer: tile, step; steps issued
  auto set_fill = [&](int t) __attribute__((always_inline)) {
    const int m0 = (t / gridN) * 256, n0 = (t % gridN) * 256;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int ra = m0 + lrow + 16 * i, rb = n0 + lrow + 16 * i;
      va[i] = ra < a.M ? (unsigned)(((long)ra * a.lda + lc * 8) * 2) : BUF_OOB;
      vb[i] = rb < a.N ? (unsigned)(((long)rb * a.ldb + lc * 8) * 2) : BUF_OOB;
    }
  };
  auto piece = [&](int q, int ks) __attribute__((always_inline)) {   // piece q (A 0..3, B 4..7) of step ks into slot nfill % 4
    ks = ks < nkr ? ks : 0;
    char* d = smem + (nfill & 3) * W4_SLOT + (q < 4 ? 0 : W4_OP) + (w * 64 + 16 * (q & 3)) * 64;
    const unsigned v = q < 4 ? va[q & 3] : vb[q & 3];
    const unsigned o = (ks * 32 + lc * 8 < a.K && v != BUF_OOB) ? v + ks * 64 : BUF_OOB;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(q < 4 ? rA : rB, (__attribute__((address_space(3))) void*)d, 16, o, 0, 0, 0);
  };
  auto fill_next = [&]() __attribute__((always_inline)) {   // (past the walk: the last tile's step 0 again)
    ++nfill;
    if (dt < tiles && ++dks == nk) {
      dks = 0;
      if (dt + nwg < tiles) {
        dt += nwg;
        set_fill(dt);
      } else {
        dt = tiles;
      }
    }
  };
  set_fill(dt);
#pragma unroll 1
  for (int s = 0; s < W4_NS; ++s) {
    const int ks = dks;
#pragma unroll
    for (int q = 0; q < 8; ++q) piece(q, ks);
    fill_next();
  }

  f32x4 acc[8][8];
  bf16x8 fa[2][8], fb[2][8];
  auto read_frag_at = [&](auto P, int q, int sl) __attribute__((always_inline)) {   // fragments q of the step in slot sl % 4
    const char* sa = smem + (sl & 3) * W4_SLOT;
    fa[P][q] = *reinterpret_cast<const bf16x8*>(sa + w4_swz(wr * 128 + q * 16 + fr, fg));
    fb[P][q] = *reinterpret_cast<const bf16x8*>(sa + W4_OP + w4_swz(wc * 128 + q * 16 + fr, fg));
  };
  auto read_frag = [&](auto P, int q, bool zero) __attribute__((always_inline)) {   // fragments q of the step in slot (nfill + 1) % 4
    const char* sa = zero ? smem + W4_NS * W4_SLOT : smem + ((nfill + 1) & 3) * W4_SLOT;
    const char* sb = zero ? smem + W4_NS * W4_SLOT : sa + W4_OP;
    fa[P][q] = *reinterpret_cast<const bf16x8*>(sa + w4_swz(wr * 128 + q * 16 + fr, fg));
    fb[P][q] = *reinterpret_cast<const bf16x8*>(sb + w4_swz(wc * 128 + q * 16 + fr, fg));
  };
  // step 0's fragments
  vm_wait(24);
  __builtin_amdgcn_s_barrier();
  {
    const char* sa = smem;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      fa[0][q] = *reinterpret_cast<const bf16x8*>(sa + w4_swz(wr * 128 + q * 16 + fr, fg));
      fb[0][q] = *reinterpret_cast<const bf16x8*>(sa + W4_OP + w4_swz(wc * 128 + q * 16 + fr, fg));
    }
  }
  // one step: fill step g+4 into g's slot, read g+1's fragments, g's 64 MFMAs (C: g's register set)
  auto step = [&](auto C, bool zn) __attribute__((always_inline)) {   // (zn: the next step is a padding step)
    constexpr int X = 1 - decltype(C)::value;
    const int ks = dks;
    static_for<0, 8>([&](auto q) __attribute__((always_inline)) {
      piece(q, ks);
      read_frag(IC<X>{}, q, zn);
#pragma unroll
      for (int j = 0; j < 8; ++j) w4_mfma(acc[q][j], fb[C][j], fa[C][q]);
      if (w4_ilv) __builtin_amdgcn_sched_barrier(0);   // (W4_ILV: each group's piece and reads beside its MFMAs)
    });
    fill_next();
  };
  int st = 0;   // store instructions of the last epilogue (younger than the fills of a tile's first three steps)
  // step ks of a tile: step g+1 landed (younger: steps g+2, g+3 and, for a tile's first three steps, the last
  // epilogue's stores); this wave's step-g fragments are in registers (every wave's, after the barrier)
  auto sync = [&](int ks) __attribute__((always_inline)) {
    if (ks < 3) vm_wait(16 + st);
    else vm_wait(16);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };
  // one tile: an even number of steps (K padded with zero chunks to a multiple of 64: the accumulators start at
  // +0 and a zero product adds exactly nothing, so C is unchanged) alternating fragment sets 0 and 1; its last
  // step reads the next tile's first fragments (already landed: the stream is continuous) into set 0
  auto tile_body = [&](int t) __attribute__((always_inline)) {
    const int m0 = (t / gridN) * 256, n0 = (t % gridN) * 256;
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    w4_pad();
#pragma unroll 1
    for (int ks = 0; ks < nk; ks += 2) {
      sync(ks);
      step(IC<0>{}, ks + 1 >= nkr);
      __builtin_amdgcn_sched_barrier(0);
      sync(ks + 1);
      step(IC<1>{}, false);
      __builtin_amdgcn_sched_barrier(0);
    }
    __builtin_amdgcn_sched_barrier(0);
    w4_pad();   // (the last MFMAs' results, before the epilogue reads the accumulators)
    // ---- epilogue: the 256p kernel's, once per 64-column half of the wave's quarter (16-B nt stores of 8
    // columns; BN partial sums per 128 rows, the same reduction tree, so C and the sums are bitwise its)
    int ns = 0;
    static_for<0, 2>([&](auto h) __attribute__((always_inline)) {
      auto get = [&](int i, int j, int r) __attribute__((always_inline)) {   // one accumulator, AGPR -> VGPR
        float v;
        asm("v_accvgpr_read_b32 %0, %1" : "=v"(v) : "a"(acc[i][4 * h + j][r]));
        return v;
      };
      ns += epilogue256_get<STATS, decltype(get), true, true>(get, a, rC, rS, m0, n0, wr, 2 * wc + h, fr, fg);
    });
    st = ns;
  };
#pragma unroll 1
  for (int t = slot; t < tiles; t += nwg) tile_body(t);
  vm_wait(0);
}

// ---------------------------------------------------------------------------------
// Persistent 256x256 NT kernel, 8 waves (two per SIMD, 128x64 each as the 256p kernel) on the 4W kernel's ring
// (gemm_nt8w_kernel; opt-in XCP_NT_8W=1 while measured): 32-deep steps through 4 LDS slots, ONE barrier per
// step, the fill one stream over the workgroup's tiles (each wave 4 LDS-DMA pieces per step).  No phase
// structure: the two waves of a SIMD interleave by themselves, one's fill issue and fragment reads beside the
// other's MFMAs.  A fragments roll (row block q's next-step fragment is read right after its last MFMA), B
// fragments are double-buffered; padding step, store counting and epilogue as gemm_nt4w_kernel.
template <bool STATS>
__global__ __launch_bounds__(512) void gemm_nt8w_kernel(NTArgs a) {
  __shared__ __attribute__((aligned(16))) char smem[W4_NS * W4_SLOT + W4_OP];
  const int gridN = (a.N + 255) / 256, gridM = (a.M + 255) / 256;
  const int tiles = gridM * gridN, nwg = gridDim.x;
  const int slot = xcd_remap(blockIdx.x, nwg);
  if (slot >= tiles) return;
  for (int i = threadIdx.x; i < W4_OP / 16; i += 512)
    reinterpret_cast<uint4*>(smem + W4_NS * W4_SLOT)[i] = make_uint4(0u, 0u, 0u, 0u);
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = w >> 2, wc = w & 3;
  const int fr = lane & 15, fg = lane >> 4;
  const int nkr = (a.K + 31) / 32, nk = (nkr + 1) & ~1;
  const __amdgpu_buffer_rsrc_t rA = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(a.A), (short)0, BUF_RECORDS,
                                                                       BUF_DWORD3);
  const __amdgpu_buffer_rsrc_t rB = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(a.B), (short)0, BUF_RECORDS,
                                                                       BUF_DWORD3);
  const __amdgpu_buffer_rsrc_t rC = __builtin_amdgcn_make_buffer_rsrc(a.C, (short)0, BUF_RECORDS, BUF_DWORD3);
  const __amdgpu_buffer_rsrc_t rS = __builtin_amdgcn_make_buffer_rsrc(STATS ? (void*)a.stats : a.C, (short)0,
                                                                       BUF_RECORDS, BUF_DWORD3);
  // ---- the fill stream: wave w loads rows w*32 .. w*32+31 of both operands, 2 pieces of 16 rows each
  const int lrow = w * 32 + (lane >> 2);
  const int lc = (lane & 3) ^ w4_f(lane >> 4);
  unsigned va[2], vb[2];
  int dt = slot, dks = 0, nfill = 0;
  auto set_fill = [&](int t) __attribute__((always_inline)) {
    const int m0 = (t / gridN) * 256, n0 = (t % gridN) * 256;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int ra = m0 + lrow + 16 * i, rb = n0 + lrow + 16 * i;
      va[i] = ra < a.M ? (unsigned)(((long)ra * a.lda + lc * 8) * 2) : BUF_OOB;
      vb[i] = rb < a.N ? (unsigned)(((long)rb * a.ldb + lc * 8) * 2) : BUF_OOB;
    }
  };
  auto piece = [&](int q, int ks) __attribute__((always_inline)) {   // piece q (A 0..1, B 2..3) into slot nfill % 4
    ks = ks < nkr ? ks : 0;
    char* d = smem + (nfill & 3) * W4_SLOT + (q < 2 ? 0 : W4_OP) + (w * 32 + 16 * (q & 1)) * 64;
    const unsigned v = q < 2 ? va[q & 1] : vb[q & 1];
    const unsigned o = (ks * 32 + lc * 8 < a.K && v != BUF_OOB) ? v + ks * 64 : BUF_OOB;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(q < 2 ? rA : rB, (__attribute__((address_space(3))) void*)d, 16, o, 0, 0, 0);
  };
  auto fill_next = [&]() __attribute__((always_inline)) {
    ++nfill;
    if (dt < tiles && ++dks == nk) {
      dks = 0;
      if (dt + nwg < tiles) {
        dt += nwg;
        set_fill(dt);
      } else {
        dt = tiles;
      }
    }
  };
  set_fill(dt);
#pragma unroll 1
  for (int s = 0; s < W4_NS; ++s) {
    const int ks = dks;
#pragma unroll
    for (int q = 0; q < 4; ++q) piece(q, ks);
    fill_next();
  }
  f32x4 acc[8][4];
  bf16x8 fa[8], fb[2][4];
  auto abase = [&](bool zero) __attribute__((always_inline)) {   // the step in slot (nfill + 1) % 4, or the zero block
    return zero ? smem + W4_NS * W4_SLOT : smem + ((nfill + 1) & 3) * W4_SLOT;
  };
  vm_wait(12);
  __builtin_amdgcn_s_barrier();
#pragma unroll
  for (int q = 0; q < 8; ++q) fa[q] = *reinterpret_cast<const bf16x8*>(smem + w4_swz(wr * 128 + q * 16 + fr, fg));
#pragma unroll
  for (int j = 0; j < 4; ++j)
    fb[0][j] = *reinterpret_cast<const bf16x8*>(smem + W4_OP + w4_swz(wc * 64 + j * 16 + fr, fg));
  auto step = [&](auto C, bool zn) __attribute__((always_inline)) {   // (zn: the next step is a padding step)
    constexpr int X = 1 - decltype(C)::value;
    const int ks = dks;
    const char* sa = abase(zn);
    const char* sb = zn ? sa : sa + W4_OP;
    static_for<0, 8>([&](auto q) __attribute__((always_inline)) {
      if constexpr (q < 4) piece(q, ks);
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc[q][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[C][j], fa[q], acc[q][j], 0, 0, 0);
      fa[q] = *reinterpret_cast<const bf16x8*>(sa + w4_swz(wr * 128 + q * 16 + fr, fg));
      if constexpr (q < 4) fb[X][q] = *reinterpret_cast<const bf16x8*>(sb + w4_swz(wc * 64 + q * 16 + fr, fg));
    });
    fill_next();
  };
  int st = 0;   // store instructions of the last epilogue (younger than the fills of a tile's first three steps)
  auto sync = [&](int ks) __attribute__((always_inline)) {
    if (ks < 3) vm_wait(8 + st);
    else vm_wait(8);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };
#pragma unroll 1
  for (int t = slot; t < tiles; t += nwg) {
    const int m0 = (t / gridN) * 256, n0 = (t % gridN) * 256;
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 1
    for (int ks = 0; ks < nk; ks += 2) {
      sync(ks);
      step(IC<0>{}, ks + 1 >= nkr);
      __builtin_amdgcn_sched_barrier(0);
      sync(ks + 1);
      step(IC<1>{}, false);
      __builtin_amdgcn_sched_barrier(0);
    }
    auto get = [&](int i, int j, int r) __attribute__((always_inline)) { return acc[i][j][r]; };
    st = epilogue256_get<STATS, decltype(get), false, true>(get, a, rC, rS, m0, n0, wr, wc, fr, fg);
  }
  vm_wait(0);
}

// ---------------------------------------------------------------------------------
// Persistent 256x256 NT kernel, two MFMA phases per 64-deep K-tile and the fill issued ~1.5
// K-tiles ahead (gemm_nt256q_kernel, the default; XCP_NT_LOOP=4 keeps gemm_nt256p_kernel).
//
// The four-phase loop above pays 8 s_barrier per K-tile around 16-MFMA phases and issues the
// next K-tile's fill during the current one (its probe, profiles/r04_nt_probe.txt: MFMAs plus
// that barrier skeleton 1.31 us per K-tile against 0.86 us of MFMA issue at 2.4 GHz, the fill
// another 0.47 us exposed).  Here each wave's K-tile is
//   R0  reads B (its 64 columns) and A-top (its group's first 64 rows): 16 ds_read_b128
//   M0  32 MFMAs into acc[0..3][0..3]
//   R1  reads A-bot: 8 ds_read_b128
//   M1  32 MFMAs into acc[4..7][0..3]
// with one barrier between consecutive intervals (4 per K-tile) and wave group 1 (waves 4-7)
// one interval behind group 0, so every interval pairs one group's MFMAs with the other group's
// LDS reads and DMA issue on each SIMD.  A read interval ends with lgkmcnt(0), so the MFMA
// interval after it starts on registers that have landed.
// Ring: the two 64 KB slots of gemm_nt256p_kernel, refilled by region as soon as both groups have
// read it: a slot's A-top + B region (6 LDS-DMA instructions per wave) is free after both groups'
// R0, its A-bot region (2 per wave) after both groups' R1.  So during K-tile k a wave issues
//   R0(k): A-bot of K-tile k+1        R1(k): A-top + B of K-tile k+2
// which leaves every region 6 intervals (1.5 K-tiles) between its issue and its first reader.
// K-tiles run on across tiles (the next tile's first two K-tiles are issued during this tile's
// last two) and a finished tile's epilogue is split over the next tile's read intervals: rows
// 0-63 of each group (acc[0..3]) are stored and zeroed in R0, rows 64-127 (acc[4..7]) and the BN
// statistics row in R1 -- beside the other group's MFMAs.
// Every wave waits for its own fill with one counted vmcnt per region: the count is the number of
// VMEM instructions the wave issued after the awaited region (epilogue stores are always issued,
// masked lanes by an out-of-range offset), so each wait retires exactly that region; wave 0's
// tile-queue fetch can only add a younger instruction (a stricter wait).  Needs K > 64.
template <bool STATS, int H>
XCP_DEV void epilogue256_half(f32x4 (&acc)[8][4], const NTArgs& a, __amdgpu_buffer_rsrc_t rC,
                              __amdgpu_buffer_rsrc_t rS, int m0, int n0, int wr, int wc, int fr, int fg,
                              float (&red)[2]) {
  const int bm = m0 / 256, stat_rows = (a.M + 127) / 128;
  const int mrow = m0 + wr * 128 + fr;
  const int ncol = n0 + wc * 64;
  const bool odd = fg & 1;
  float s1[16], s2[16];
#pragma unroll
  for (int q = 0; q < 16; ++q) s1[q] = s2[q] = 0.f;
  const int c0 = ncol + (odd ? 16 + (fg - 1) * 4 : fg * 4);
  static_for<4 * H, 4 * H + 4>([&](auto i) {
    const int m = mrow + i * 16;
    const bool mok = m < a.M;
    uint2 pc[4];
    static_for<0, 4>([&](auto j) {
      pc[j] = make_uint2(pk_bf16(acc[i][j][0], acc[i][j][1]), pk_bf16(acc[i][j][2], acc[i][j][3]));
      const bf16x4 q = __builtin_bit_cast(bf16x4, pc[j]);
      if constexpr (STATS) {   // (branch-free: rows past M add zero)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float f = mok ? (float)q[r] : 0.f;
          s1[j * 4 + r] += f;
          s2[j * 4 + r] = fmaf(f, f, s2[j * 4 + r]);
        }
      }
      acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    });
    const uint2 snd0 = odd ? pc[0] : pc[1], snd1 = odd ? pc[2] : pc[3];
    uint2 rc0, rc1;
    rc0.x = __shfl_xor(snd0.x, 16, 64);
    rc0.y = __shfl_xor(snd0.y, 16, 64);
    rc1.x = __shfl_xor(snd1.x, 16, 64);
    rc1.y = __shfl_xor(snd1.y, 16, 64);
    const uint4 st0 = odd ? make_uint4(rc0.x, rc0.y, pc[1].x, pc[1].y) : make_uint4(pc[0].x, pc[0].y, rc0.x, rc0.y);
    const uint4 st1 = odd ? make_uint4(rc1.x, rc1.y, pc[3].x, pc[3].y) : make_uint4(pc[2].x, pc[2].y, rc1.x, rc1.y);
    const unsigned rowb = (unsigned)((long)m * a.ldc * 2);
    const unsigned o0 = (mok && c0 < a.N) ? rowb + (unsigned)c0 * 2 : BUF_OOB;
    const unsigned o1 = (mok && c0 + 32 < a.N) ? rowb + (unsigned)(c0 + 32) * 2 : BUF_OOB;
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(i32x4, st0), rC, (int)o0, 0, 0);
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(i32x4, st1), rC, (int)o1, 0, 0);
  });
  if constexpr (STATS) {   // this half's column sums, reduced over the wave as epilogue256_get does
    float u[16], v8[8], v4[4];
    const bool b3 = fr & 8, b2 = fr & 4, b1 = fr & 2, b0 = fr & 1;
#pragma unroll
    for (int q = 0; q < 16; ++q) u[q] = (b3 ? s2[q] : s1[q]) + __shfl_xor(b3 ? s1[q] : s2[q], 8, 64);
#pragma unroll
    for (int q = 0; q < 8; ++q) v8[q] = (b2 ? u[8 + q] : u[q]) + __shfl_xor(b2 ? u[q] : u[8 + q], 4, 64);
#pragma unroll
    for (int q = 0; q < 4; ++q) v4[q] = (b1 ? v8[4 + q] : v8[q]) + __shfl_xor(b1 ? v8[q] : v8[4 + q], 2, 64);
#pragma unroll
    for (int q = 0; q < 2; ++q) red[q] += (b0 ? v4[2 + q] : v4[q]) + __shfl_xor(b0 ? v4[q] : v4[2 + q], 1, 64);
    if constexpr (H == 1) {
      const int col = ncol + ((fr & 7) >> 1) * 16 + fg * 4 + (fr & 1) * 2;
      const int srow = bm * 2 + wr;
      const unsigned so = (srow < stat_rows && col < a.N)
                              ? (unsigned)((((long)srow * 2 + (fr >> 3)) * a.N + col) * 4) : BUF_OOB;
      __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(i32x2, make_float2(red[0], red[1])), rS, (int)so, 0, 0);
      red[0] = red[1] = 0.f;
    }
  }
}

// s_waitcnt vmcnt(n) for the counts gemm_nt256q_kernel forms (steady state 8 first; any other
// value waits for everything, which is only ever stricter)
XCP_DEV void vm_wait_q(int n) {
#define XCP_VMQ(k) if (n == k) { asm volatile("s_waitcnt vmcnt(" #k ")" ::: "memory"); return; }
  XCP_VMQ(8) XCP_VMQ(16) XCP_VMQ(17) XCP_VMQ(18) XCP_VMQ(19) XCP_VMQ(24) XCP_VMQ(25) XCP_VMQ(2)
#undef XCP_VMQ
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

XCP_DEV void nt_barrier() {
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}

template <bool STATS>
__global__ __launch_bounds__(512) void gemm_nt256q_kernel(NTArgs a) {
  constexpr int EA = 8, EB = 8 + (STATS ? 1 : 0);   // epilogue stores per wave in R0 / in R1
  __shared__ __attribute__((aligned(16))) char smem[2 * K_SLOT + 16];
  int* const s_next = reinterpret_cast<int*>(smem + 2 * K_SLOT);
  int* const tq = a.tqs > 0 ? g_nt_tq + (a.tqs - 1) : nullptr;
  const int gridN = (a.N + 255) / 256, gridM = (a.M + 255) / 256;
  const int tiles = gridM * gridN, nwg = gridDim.x;
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = w >> 2, wc = w & 3;
  const int arow = (w < 4 ? 16 * w : 128 + 16 * (w - 4));
  const int brow = 64 * (w >> 1) + 16 * (w & 1);
  const int lr = lane >> 3;
  // per lane: the rows it fills of each half-tile (wave base + i * 8 + lr) and the 16-B chunk of the
  // 128-B row (XOR-swizzled by (row >> 1) & 7 = (i * 4 + lr / 2) & 7: every base is a multiple of 16);
  // the tile only adds a scalar row offset, so the per-lane part of each offset is tile-independent
  const int kc8[2] = {((lane & 7) ^ ((lr >> 1) & 7)) * 8, ((lane & 7) ^ ((4 + (lr >> 1)) & 7)) * 8};
  auto hbase = [&](int h) {   // wave-uniform first row of half-tile h this wave fills
    return (h == 0 || h == 3) ? arow + (h == 3 ? 64 : 0) : brow + (h == 2 ? 32 : 0);
  };
  unsigned lpart[4][2];
#pragma unroll
  for (int h = 0; h < 4; ++h)
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const bool isA = (h == 0 || h == 3);
      lpart[h][i] = (unsigned)(((long)(hbase(h) + i * 8 + lr) * (isA ? a.lda : a.ldb) + kc8[i]) * 2);
    }
  const __amdgpu_buffer_rsrc_t rA = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(a.A), (short)0, BUF_RECORDS,
                                                                       BUF_DWORD3);
  const __amdgpu_buffer_rsrc_t rB = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(a.B), (short)0, BUF_RECORDS,
                                                                       BUF_DWORD3);
  const __amdgpu_buffer_rsrc_t rC = __builtin_amdgcn_make_buffer_rsrc(a.C, (short)0, BUF_RECORDS, BUF_DWORD3);
  const __amdgpu_buffer_rsrc_t rS = __builtin_amdgcn_make_buffer_rsrc(STATS ? (void*)a.stats : a.C, (short)0,
                                                                       BUF_RECORDS, BUF_DWORD3);
  // half-tile h of K-tile kt of tile tt into ring slot sl: 2 instructions
  auto issue = [&](int tt, int h, int kt, int sl) {
    const bool isA = (h == 0 || h == 3);
    const int row0 = hbase(h);
    const int tb = isA ? (tt / gridN) * 256 : (tt % gridN) * 256;   // (uniform)
    const unsigned tofs = (unsigned)((long)tb * (isA ? a.lda : a.ldb) * 2);
    char* d = smem + sl * K_SLOT + (isA ? 0 : K_OP) + row0 * 128;
    const int kb = kt * 64;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const bool ok = tb + row0 + i * 8 + lr < (isA ? a.M : a.N) && kb + kc8[i] < a.K;
      const unsigned o = ok ? lpart[h][i] + tofs + kb * 2 : BUF_OOB;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(isA ? rA : rB, (__attribute__((address_space(3))) void*)(d + i * 1024),
                                               16, o, 0, 0, 0);
    }
  };
  auto issue_atb = [&](int tt, int kt, int sl) {   // 6 instructions
    issue(tt, 0, kt, sl);
    issue(tt, 1, kt, sl);
    issue(tt, 2, kt, sl);
  };

  int t = xcd_remap(blockIdx.x, nwg);
  if (t >= tiles) return;
  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  float red[2] = {0.f, 0.f};
  const int nk = (a.K + 63) / 64;
  const int fr = lane & 15, fg = lane >> 4;
  bf16x8 af[4][2], bf[4][2];
  // the next tile: known now on the static walk; with the tile queue fetched at each tile's start
  // and published at K-tile nk-2
  int tn = t + nwg;
  bool more = !tq && tn < tiles;
  // prologue: A-top + B of K-tiles 0 and 1, A-bot of 0; wait for K-tile 0's A-top + B
  issue_atb(t, 0, 0);
  issue(t, 3, 0, 0);
  issue_atb(t, 1, 1);
  vm_wait_q(8);
  nt_barrier();
  if (wr == 1) nt_barrier();

  int sb = 0;              // ring slot of this tile's K-tile 0
  int pt = 0;              // the finished tile whose epilogue runs during K-tile 0 (when follow)
  bool follow = false;     // this tile follows another one of this workgroup
  unsigned nxt = 0;
  int kt = 0;
  while (true) {
    const int sl = (sb + kt) & 1;
    const char* sa = smem + sl * K_SLOT;
    const char* sbp = sa + K_OP;
    const bool last = kt + 1 == nk;
    const bool e0 = follow && kt == 0;           // epilogue halves in this K-tile's R0 / R1
    const bool e_prev = follow && kt == 1;       // ... in the previous K-tile's
    const bool ex1 = !last || more;              // K-tile k+1 exists (this tile's or the next one's)
    // ---- R0: epilogue rows 0-63, B + A-top fragments, A-bot fill of K-tile k+1
    if (e0) epilogue256_half<STATS, 0>(acc, a, rC, rS, (pt / gridN) * 256, (pt % gridN) * 256, wr, wc, fr, fg, red);
    if (kt == 0 && tq && tid == 0)
      asm volatile("global_atomic_add %0, %1, %2, off sc0" : "=v"(nxt) : "v"(tq), "v"(1u) : "memory");
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
#pragma unroll
      for (int j = 0; j < 4; ++j)
        bf[j][ks] = *reinterpret_cast<const bf16x8*>(sbp + swz(wc * 64 + j * 16 + fr, ks * 4 + fg));
#pragma unroll
      for (int i = 0; i < 4; ++i)
        af[i][ks] = *reinterpret_cast<const bf16x8*>(sa + swz(wr * 128 + i * 16 + fr, ks * 4 + fg));
    }
    if (!last) issue(t, 3, kt + 1, sl ^ 1);
    else if (more) issue(tn, 3, 0, sl ^ 1);
    // A-bot of K-tile k (issued in R0(k-1)) is followed by: R1(k-1)'s epilogue half and A-top + B of
    // k+1, this R0's epilogue half and A-bot of k+1
    const int c_ab = (e_prev ? EB : 0) + (ex1 ? 8 : 0) + (e0 ? EA : 0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (wr == 1) vm_wait_q(c_ab);
    nt_barrier();
    // ---- M0
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[j][ks], af[i][ks], acc[i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
    if (wr == 0) vm_wait_q(c_ab);
    if (tq && kt == nk - 2 && tid == 0) {   // publish the next tile (the fetch has retired)
      if (nk == 2) vm_wait_q(2);              // (K-tile 0: only A-bot of K-tile 1 follows the fetch)
      asm volatile("" : "+v"(nxt));
      *s_next = (int)nxt;
      if ((int)nxt == tiles - 1) __hip_atomic_store(tq, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    nt_barrier();
    // ---- R1: epilogue rows 64-127 + statistics, A-bot fragments, A-top + B fill of K-tile k+2
    if (tq && kt == nk - 2) {
      tn = nwg + __builtin_amdgcn_readfirstlane(*s_next);
      more = tn < tiles;
    }
    if (e0) epilogue256_half<STATS, 1>(acc, a, rC, rS, (pt / gridN) * 256, (pt % gridN) * 256, wr, wc, fr, fg, red);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < 4; ++i)
        af[i][ks] = *reinterpret_cast<const bf16x8*>(sa + swz(wr * 128 + 64 + i * 16 + fr, ks * 4 + fg));
    const bool ex2 = kt + 2 < nk || more;        // K-tile k+2 exists
    if (kt + 2 < nk) issue_atb(t, kt + 2, sl);
    else if (more) issue_atb(tn, kt + 2 - nk, sl);
    // A-top + B of K-tile k+1 (issued in R1(k-1)) is followed by: this K-tile's two epilogue halves,
    // A-bot of k+1 and A-top + B of k+2
    const int c_atb = (e0 ? EA + EB : 0) + (ex1 ? 2 : 0) + (ex2 ? 6 : 0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (wr == 1 && ex1) vm_wait_q(c_atb);
    nt_barrier();
    // ---- M1
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[4 + i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[j][ks], af[i][ks], acc[4 + i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
    if (wr == 0 && ex1) vm_wait_q(c_atb);
    nt_barrier();
    if (!last) {
      ++kt;
      continue;
    }
    if (!more) break;
    // next tile: its K-tiles 0 and 1 are in flight, this one's epilogue runs in its K-tile 0
    pt = t;
    t = tn;
    sb = (sb + nk) & 1;
    kt = 0;
    follow = true;
    tn = t + nwg;
    more = !tq && tn < tiles;
  }
  if (wr == 0) nt_barrier();   // (group 1 ran one barrier behind)
  const int m0 = (t / gridN) * 256, n0 = (t % gridN) * 256;
  epilogue256_half<STATS, 0>(acc, a, rC, rS, m0, n0, wr, wc, fr, fg, red);
  epilogue256_half<STATS, 1>(acc, a, rC, rS, m0, n0, wr, wc, fr, fg, red);
}

// ---------------------------------------------------------------------------------
// Weight gradient: P[s][n][k] = sum_{m in split s} G[m][n] * X[m][k]
// G: [M][ldg] (output-gradient pixel rows), X: [M][ldx] (layer-input pixel rows).
// Both operands are pixel-major, so the reduction index m is the slow memory
// dimension: tiles are staged [m][col] in LDS and bf16 fragments are read with
// ds_read_b64_tr_b16 (4 m-rows x 16 cols per 16-lane group, transposed).
constexpr int TBM = 32;                      // m rows per stage
constexpr int TPITCH = 128 * 2 + 32;         // bf16 LDS row pitch (bytes): pitch/4 = 8 (mod 64)

struct TNArgs {
  const void* G; long ldg;
  const void* X; long ldx;
  float* P;                // [S][N][K] fp32 partials
  int M, N, K, S, rows_per_split;
  Gather gx;               // gather of the X operand rows / columns
  int xalign;              // 256x256 kernel: workgroup b = split (b / 8 / tiles) * 8 + b % 8, tile b / 8 % tiles
};

template <typename T, int GM>
__global__ __launch_bounds__(NT) void gemm_tn_kernel(TNArgs a) {
  // tile: 128 (n) x 128 (k); stage: 32 m-rows of G[., n0:n0+128] and X[., k0:k0+128]
  constexpr int EPC = GT<T>::EPC;
  constexpr int PITCH = (sizeof(T) == 2) ? TPITCH : (128 * 4 + 16);
  constexpr int STG = TBM * PITCH;
  __shared__ __attribute__((aligned(16))) char smem[4 * STG];

  const int gridN = (a.N + 127) / 128, gridK = (a.K + 127) / 128;
  const int tiles = gridN * gridK;
  // logical ids of one row split are contiguous and land on one XCD, so the
  // split's G / X rows are fetched from HBM once and re-served by that XCD's L2
  const int id = xcd_remap(blockIdx.x, gridDim.x);
  const int s = id / tiles, t = id % tiles;
  const int bn = t / gridK, bk = t % gridK;
  const int n0 = bn * 128, k0 = bk * 128;
  const int mbeg = s * a.rows_per_split;
  const int mend = min(a.M, mbeg + a.rows_per_split);
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wm = w >> 1, wn = w & 1;            // wave tile: n rows wm*64.., k cols wn*64..
  const T* G = reinterpret_cast<const T*>(a.G);
  const T* X = reinterpret_cast<const T*>(a.X);

  // staging: each operand stage = 32 rows x 128 cols = 32 x (128/EPC) chunks
  constexpr int CPR = 128 / EPC;            // 16 (bf16) or 32 (f32) chunks per row
  constexpr int LPT = TBM * CPR / NT;       // loads per thread per operand: 2 or 4
  uint4 rg[LPT], rx[LPT];
  int srow[LPT], schk[LPT];
#pragma unroll
  for (int i = 0; i < LPT; ++i) {
    const int q = tid + NT * i;
    srow[i] = q / CPR;
    schk[i] = q % CPR;
  }
  auto gload = [&](int mb) {
#pragma unroll
    for (int i = 0; i < LPT; ++i) {
      const int m = mb + srow[i];
      const int n = n0 + schk[i] * EPC, k = k0 + schk[i] * EPC;
      const bool mok = m < mend;
      rg[i] = (mok && n < a.N) ? *reinterpret_cast<const uint4*>(G + (long)m * a.ldg + n) : make_uint4(0, 0, 0, 0);
      const RowInfo xr = row_info<GM>(a.gx, m, mend);
      const long xo = (xr.ok && k < a.K) ? chunk_off<GM>(a.gx, xr, a.ldx, k) : -1;
      rx[i] = xo >= 0 ? *reinterpret_cast<const uint4*>(X + xo) : make_uint4(0, 0, 0, 0);
    }
  };
  auto swrite = [&](int buf) {
    char* sg = smem + buf * 2 * STG;
    char* sx = sg + STG;
#pragma unroll
    for (int i = 0; i < LPT; ++i) {
      *reinterpret_cast<uint4*>(sg + srow[i] * PITCH + schk[i] * 16) = rg[i];
      *reinterpret_cast<uint4*>(sx + srow[i] * PITCH + schk[i] * 16) = rx[i];
    }
  };

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int fr = lane & 15, fg = lane >> 4;
  const int q4 = fr >> 2, p4 = fr & 3;          // tr-read: lane 4q+p -> row q, cols 4p..4p+3
  const int nst = (mend - mbeg + TBM - 1) / TBM;
  if (nst > 0) {
    gload(mbeg);
    swrite(0);
  }
  __syncthreads();
  for (int st = 0; st < nst; ++st) {
    if (st + 1 < nst) gload(mbeg + (st + 1) * TBM);
    const char* sg = smem + (st & 1) * 2 * STG;
    const char* sx = sg + STG;
    if constexpr (sizeof(T) == 2) {
      // MFMA k-slots of lane group g: m rows {4g..4g+3} (elements 0-3) and {16+4g..} (4-7)
      bf16x8 af[4], bfr[4];
#pragma unroll
      for (int t4 = 0; t4 < 4; ++t4) {
        const int ncol = wm * 64 + t4 * 16 + p4 * 4;
        const int kcol = wn * 64 + t4 * 16 + p4 * 4;
        bf16x4 a0 = ds_read_tr(sg + (4 * fg + q4) * PITCH + ncol * 2);
        bf16x4 a1 = ds_read_tr(sg + (16 + 4 * fg + q4) * PITCH + ncol * 2);
        bf16x4 b0 = ds_read_tr(sx + (4 * fg + q4) * PITCH + kcol * 2);
        bf16x4 b1 = ds_read_tr(sx + (16 + 4 * fg + q4) * PITCH + kcol * 2);
        af[t4] = bf16x8{a0[0], a0[1], a0[2], a0[3], a1[0], a1[1], a1[2], a1[3]};
        bfr[t4] = bf16x8{b0[0], b0[1], b0[2], b0[3], b1[0], b1[1], b1[2], b1[3]};
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    } else {
      // fp32: 8 MFMA steps of 4 m-rows; lane group g holds m row 4*step + g
#pragma unroll
      for (int e = 0; e < TBM / 4; ++e) {
        const int mr = 4 * e + fg;
        float av[4], bv[4];
#pragma unroll
        for (int t4 = 0; t4 < 4; ++t4) {
          av[t4] = *reinterpret_cast<const float*>(sg + mr * PITCH + (wm * 64 + t4 * 16 + fr) * 4);
          bv[t4] = *reinterpret_cast<const float*>(sx + mr * PITCH + (wn * 64 + t4 * 16 + fr) * 4);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[i], bv[j], acc[i][j], 0, 0, 0);
      }
    }
    if (st + 1 < nst) swrite((st + 1) & 1);
    __syncthreads();
  }
  // write partial slab P[s][n][k]: acc[i][j][r] = C[n = wm*64+i*16+fg*4+r][k = wn*64+j*16+fr]
  float* P = a.P + (long)s * a.N * a.K;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int n = n0 + wm * 64 + i * 16 + fg * 4 + r;
      if (n >= a.N) continue;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int k = k0 + wn * 64 + j * 16 + fr;
        if (k < a.K) P[(long)n * a.K + k] = acc[i][j][r];
      }
    }
}


// ---------------------------------------------------------------------------------
// 256x256 bf16 weight-gradient kernel: P[s][n][k] = sum_{m in split s} G[m][n] X[m][k].
// 8 waves (2 n-groups x 4 k-groups, wave tile 128 n x 64 k), staggered by one barrier as
// gemm_nt256k64_kernel.  The reduction index m is the ROW index of both operands, so a
// step is 32 m-rows of each (512-B slab rows: every LDS-DMA instruction moves whole
// 128-B lines at any step depth; 16-B chunk c of row m stored at c ^ ((m & 7) << 1),
// which makes the transposed ds_read_b64_tr_b16 fragment reads conflict-free).
// Both operands stream from HBM (nothing L2-resident, unlike the NT weights), so the
// kernel is bound by bytes in flight per CU: a ring of 5 steps x 32 KB (all 160 KB of
// LDS) keeps 3 steps (~96 KB) in flight.  Step s is two phases:
//   A (n-top): reads X frags + G n-top   issues G(s+3)   retires G/X(s+1)
//   B (n-bot): reads G n-bot             issues X(s+3)
// A step's data is retired one phase before the first barrier its readers pass; the
// slot of s+3 is the slot of s-2, last read >= 3 phases earlier.
typedef unsigned long long u64;
typedef u64 u64x2 __attribute__((ext_vector_type(2)));

XCP_DEV unsigned lds_addr(const char* p) {
  return (unsigned)(size_t)(const __attribute__((address_space(3))) char*)(p);
}
// ds_read_b64_tr_b16 outside the compiler's view (no implicit vmcnt(0) ahead of it, and no
// implicit lgkmcnt before the result's use: lds_fence below must retire it first)
XCP_DEV u64 ds_read_tr_asm(const char* p) {
  u64 v;
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(v) : "v"(lds_addr(p)) : "memory");
  return v;
}
// s_waitcnt lgkmcnt(0) that the listed fragments (2 x 64 bit each) depend on, so no use of
// them can be scheduled ahead of it; lds_pin orders more fragments after that wait
XCP_DEV void lds_fence(u64 (&a)[2], u64 (&b)[2], u64 (&c)[2], u64 (&d)[2]) {
  asm volatile("s_waitcnt lgkmcnt(0)"
               : "+v"(a[0]), "+v"(a[1]), "+v"(b[0]), "+v"(b[1]), "+v"(c[0]), "+v"(c[1]), "+v"(d[0]), "+v"(d[1])
               :
               : "memory");
}
XCP_DEV void lds_pin(u64 (&a)[2], u64 (&b)[2], u64 (&c)[2], u64 (&d)[2]) {
  asm volatile("" : "+v"(a[0]), "+v"(a[1]), "+v"(b[0]), "+v"(b[1]), "+v"(c[0]), "+v"(c[1]), "+v"(d[0]), "+v"(d[1]));
}

constexpr int T_HALF = 32 * 512;               // one operand, one step (16 KB)
constexpr int T_STEP = 2 * T_HALF;
constexpr int T_RING = 5;

XCP_DEV int tswz(int m, int col) {             // byte offset of bf16 column col of slab row m
  return m * 512 + ((((col >> 3) ^ ((m & 7) << 1))) << 4) + (col & 7) * 2;
}

template <bool BUF>
__global__ __launch_bounds__(512) void gemm_tn256_kernel(TNArgs a) {
  __shared__ __attribute__((aligned(16))) char smem[T_RING * T_STEP];
  const int gridN = (a.N + 255) / 256, gridK = (a.K + 255) / 256;
  const int tiles = gridN * gridK;
  // one split's tiles on one XCD, where its row panels are shared through L2.  xalign: workgroups go
  // to the XCDs round-robin (b % 8), so split (q / tiles) * 8 + b % 8 takes every tile q % tiles of
  // XCD b % 8's slot row q / tiles -- whole splits per XCD (the grid is padded to 8 splits per slot
  // row; the padding workgroups return at once).  Otherwise consecutive remapped ids share an XCD,
  // and a split whose tiles straddle two ranges is read by both XCDs.
  int sp, t;
  if (a.xalign) {
    const int q = blockIdx.x >> 3;
    sp = (q / tiles) * 8 + (blockIdx.x & 7);
    t = q % tiles;
    if (sp >= a.S) return;
  } else {
    const int id = xcd_remap(blockIdx.x, gridDim.x);
    sp = id / tiles;
    t = id % tiles;
  }
  const int n0 = (t / gridK) * 256, k0 = (t % gridK) * 256;
  const int mbeg = sp * a.rows_per_split;
  const int mend = min(a.M, mbeg + a.rows_per_split);
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);   // wave-uniform: LDS-DMA destinations (M0) from SGPRs
  const int wr = w >> 2, wc = w & 3;
  const bf16* G = reinterpret_cast<const bf16*>(a.G);
  const bf16* X = reinterpret_cast<const bf16*>(a.X);

  // staging: a half-step is 32 m-rows x 512 B; wave w loads rows 4w + 2i + (lane >> 5)
  // (i = 0, 1), lane writes physical chunk lane & 31 = logical chunk lc
  const int pc = lane & 31;
  int rr[2], lc[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    rr[i] = 4 * w + 2 * i + (lane >> 5);
    lc[i] = pc ^ ((rr[i] & 7) << 1);
  }
  const void* zero = g_zero16;
  asm volatile("" : "+v"(zero));
  auto glds = [](const void* p, char* dst) {
    __builtin_amdgcn_global_load_lds((const void __attribute__((address_space(1)))*)p,
                                     (void __attribute__((address_space(3)))*)dst, 16, 0, 0);
  };
  const __amdgpu_buffer_rsrc_t rG = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(a.G), (short)0, BUF_RECORDS,
                                                                       BUF_DWORD3);
  const __amdgpu_buffer_rsrc_t rX = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(a.X), (short)0, BUF_RECORDS,
                                                                       BUF_DWORD3);
  // operand isG of step st into ring slot sl
  auto issue = [&](bool isG, int st, int sl) {
    char* d = smem + sl * T_STEP + (isG ? 0 : T_HALF);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int m = mbeg + st * 32 + rr[i];
      const int col = (isG ? n0 : k0) + lc[i] * 8;
      const bool ok = m < mend && col < (isG ? a.N : a.K);
      char* dst = d + (4 * w + 2 * i) * 512;   // 1 KB = slab rows 4w+2i, +1
      if constexpr (BUF) {
        const unsigned o = ok ? (unsigned)(((long)m * (isG ? a.ldg : a.ldx) + col) * 2) : BUF_OOB;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(isG ? rG : rX, (__attribute__((address_space(3))) void*)dst, 16, o,
                                                 0, 0, 0);
      } else {
        const void* src = ok ? (isG ? (const void*)(G + (long)m * a.ldg + col)
                                    : (const void*)(X + (long)m * a.ldx + col))
                             : zero;
        glds(src, dst);
      }
    }
  };

  f32x4 acc[8][4];   // [n-frag][k-frag]: lane holds P[n = .. + fr][k = .. + 4*fg + r]
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int ns = (mend - mbeg + 31) / 32;
  // prologue: steps 0..2 in flight, step 0 retired
#pragma unroll
  for (int st = 0; st < 3; ++st)
    if (st < ns) {
      issue(true, st, st);
      issue(false, st, st);
    }
  if (ns >= 3) wait_vmcnt<8>();
  else if (ns == 2) wait_vmcnt<4>();
  else wait_vmcnt<0>();
  __builtin_amdgcn_s_barrier();
  if (wr == 1) __builtin_amdgcn_s_barrier();

  const int fr = lane & 15, fg = lane >> 4;
  const int q4 = fr >> 2, p4 = fr & 3;   // tr read: lane 4q+p reads slab row q, columns 4p..4p+3
  // fragment of 16 columns at cb: k-slots of lane group fg are slab rows {4fg..4fg+3}
  // (elements 0-3, r[0]) and 16 + {4fg..} (4-7, r[1]).  The transposed reads are issued
  // by inline asm: hipcc waits vmcnt(0) before every ds_read_tr builtin while any LDS-DMA
  // is in flight (draining the ring each phase); the counted vmcnt + barrier protocol
  // above is what orders them, and lds_fence() retires them before their first use.
  auto frag = [&](const char* slab, int cb, u64 (&r)[2]) {
    const int m0r = 4 * fg + q4;
    const int col = cb + 4 * p4;
    r[0] = ds_read_tr_asm(slab + tswz(m0r, col));
    r[1] = ds_read_tr_asm(slab + tswz(m0r + 16, col));
  };
  auto b8 = [](const u64 (&r)[2]) { return __builtin_bit_cast(bf16x8, u64x2{r[0], r[1]}); };
  u64 gr[4][2], xr[4][2];
  auto mfma4 = [&](int ih) {
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc[ih * 4 + i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b8(xr[j]), b8(gr[i]), acc[ih * 4 + i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_s_barrier();
  };
  int slot = 0, pslot = 3;   // ring slots of step s and of step s + 3
  for (int s = 0; s < ns; ++s) {
    const char* sg = smem + slot * T_STEP;
    const char* sx = sg + T_HALF;
    const bool pre = s + 3 < ns;
    // A: n-top
#pragma unroll
    for (int j = 0; j < 4; ++j) frag(sx, wc * 64 + j * 16, xr[j]);
#pragma unroll
    for (int i = 0; i < 4; ++i) frag(sg, wr * 128 + i * 16, gr[i]);
    if (pre) issue(true, s + 3, pslot);
    // retire step s+1: loads issued after X(s+1) may stay in flight
    if (pre) wait_vmcnt<6>();
    else if (s + 2 < ns) wait_vmcnt<4>();
    else wait_vmcnt<0>();
    __builtin_amdgcn_s_barrier();
    lds_fence(xr[0], xr[1], xr[2], xr[3]);
    lds_pin(gr[0], gr[1], gr[2], gr[3]);
    mfma4(0);
    // B: n-bot
#pragma unroll
    for (int i = 0; i < 4; ++i) frag(sg, wr * 128 + 64 + i * 16, gr[i]);
    if (pre) issue(false, s + 3, pslot);
    __builtin_amdgcn_s_barrier();
    lds_fence(gr[0], gr[1], gr[2], gr[3]);
    mfma4(1);
    slot = slot == T_RING - 1 ? 0 : slot + 1;
    pslot = pslot == T_RING - 1 ? 0 : pslot + 1;
  }
  if (wr == 0) __builtin_amdgcn_s_barrier();

  float* P = a.P + (long)sp * a.N * a.K;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int n = n0 + wr * 128 + i * 16 + fr;
    if (n >= a.N) continue;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int k = k0 + wc * 64 + j * 16 + 4 * fg;
      if (k < a.K) *reinterpret_cast<f32x4*>(P + (long)n * a.K + k) = acc[i][j];
    }
  }
}

// Weight-gradient kernel with ONE MFMA phase of 32 per 32-row step and the fill four steps ahead
// (gemm_tn256q_kernel, the default; XCP_TN_LOOP=1 runs gemm_tn256_kernel's two 16-MFMA phases).  Per step
// a wave reads all its fragments (X: 4 k-frags, G: 8 n-frags = 24 ds_read_b64_tr_b16) and issues
// step s+4 into the slot step s-1 left (both wave groups finished reading it two intervals earlier),
// waits lgkmcnt(0), and its 32 MFMAs run in the next interval beside the other group's reads: two
// barriers per step instead of four, and 4 x 32 KB of the 5-slot ring in flight instead of 3.
XCP_DEV void tn_vm_wait(int n) {
  if (n >= 12) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
  else if (n >= 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else if (n >= 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

template <bool BUF>
__global__ __launch_bounds__(512) void gemm_tn256q_kernel(TNArgs a) {
  __shared__ __attribute__((aligned(16))) char smem[T_RING * T_STEP];
  const int gridN = (a.N + 255) / 256, gridK = (a.K + 255) / 256;
  const int tiles = gridN * gridK;
  int sp, t;
  if (a.xalign) {
    const int q = blockIdx.x >> 3;
    sp = (q / tiles) * 8 + (blockIdx.x & 7);
    t = q % tiles;
    if (sp >= a.S) return;
  } else {
    const int id = xcd_remap(blockIdx.x, gridDim.x);
    sp = id / tiles;
    t = id % tiles;
  }
  const int n0 = (t / gridK) * 256, k0 = (t % gridK) * 256;
  const int mbeg = sp * a.rows_per_split;
  const int mend = min(a.M, mbeg + a.rows_per_split);
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = w >> 2, wc = w & 3;
  const bf16* G = reinterpret_cast<const bf16*>(a.G);
  const bf16* X = reinterpret_cast<const bf16*>(a.X);
  const int pc = lane & 31;
  int rr[2], lc[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    rr[i] = 4 * w + 2 * i + (lane >> 5);
    lc[i] = pc ^ ((rr[i] & 7) << 1);
  }
  const void* zero = g_zero16;
  asm volatile("" : "+v"(zero));
  auto glds = [](const void* p, char* dst) {
    __builtin_amdgcn_global_load_lds((const void __attribute__((address_space(1)))*)p,
                                     (void __attribute__((address_space(3)))*)dst, 16, 0, 0);
  };
  const __amdgpu_buffer_rsrc_t rG = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(a.G), (short)0, BUF_RECORDS,
                                                                       BUF_DWORD3);
  const __amdgpu_buffer_rsrc_t rX = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(a.X), (short)0, BUF_RECORDS,
                                                                       BUF_DWORD3);
  auto issue = [&](bool isG, int st, int sl) {   // 2 instructions
    char* d = smem + sl * T_STEP + (isG ? 0 : T_HALF);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int m = mbeg + st * 32 + rr[i];
      const int col = (isG ? n0 : k0) + lc[i] * 8;
      const bool ok = m < mend && col < (isG ? a.N : a.K);
      char* dst = d + (4 * w + 2 * i) * 512;
      if constexpr (BUF) {
        const unsigned o = ok ? (unsigned)(((long)m * (isG ? a.ldg : a.ldx) + col) * 2) : BUF_OOB;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(isG ? rG : rX, (__attribute__((address_space(3))) void*)dst, 16, o,
                                                 0, 0, 0);
      } else {
        const void* src = ok ? (isG ? (const void*)(G + (long)m * a.ldg + col)
                                    : (const void*)(X + (long)m * a.ldx + col))
                             : zero;
        glds(src, dst);
      }
    }
  };

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int ns = (mend - mbeg + 31) / 32;
  // prologue: steps 0..3 in flight, step 0 retired
#pragma unroll
  for (int st = 0; st < 4; ++st)
    if (st < ns) {
      issue(true, st, st);
      issue(false, st, st);
    }
  tn_vm_wait(4 * (min(ns, 4) - 1));
  __builtin_amdgcn_s_barrier();
  if (wr == 1) __builtin_amdgcn_s_barrier();

  const int fr = lane & 15, fg = lane >> 4;
  const int q4 = fr >> 2, p4 = fr & 3;
  auto frag = [&](const char* slab, int cb, u64 (&r)[2]) {
    const int m0r = 4 * fg + q4;
    const int col = cb + 4 * p4;
    r[0] = ds_read_tr_asm(slab + tswz(m0r, col));
    r[1] = ds_read_tr_asm(slab + tswz(m0r + 16, col));
  };
  auto b8 = [](const u64 (&r)[2]) { return __builtin_bit_cast(bf16x8, u64x2{r[0], r[1]}); };
  u64 gr[8][2], xr[4][2];
  int slot = 0, pslot = 4;   // ring slots of step s and of step s + 4
  for (int s = 0; s < ns; ++s) {
    const char* sg = smem + slot * T_STEP;
    const char* sx = sg + T_HALF;
    // R: every fragment of the step, step s+4's fill
#pragma unroll
    for (int j = 0; j < 4; ++j) frag(sx, wc * 64 + j * 16, xr[j]);
#pragma unroll
    for (int i = 0; i < 8; ++i) frag(sg, wr * 128 + i * 16, gr[i]);
    if (s + 4 < ns) {
      issue(true, s + 4, pslot);
      issue(false, s + 4, pslot);
    }
    lds_fence(xr[0], xr[1], xr[2], xr[3]);
    lds_pin(gr[0], gr[1], gr[2], gr[3]);
    lds_pin(gr[4], gr[5], gr[6], gr[7]);
    // step s+1 landed (this wave's part): after it, steps s+2 .. s+4 (4 instructions each, if issued)
    const int younger = 4 * (min(ns - 1, s + 4) - (s + 1));
    if (wr == 1 && s + 1 < ns) tn_vm_wait(younger);
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    // M: 32 MFMAs
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b8(xr[j]), b8(gr[i]), acc[i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
    if (wr == 0 && s + 1 < ns) tn_vm_wait(younger);
    __builtin_amdgcn_s_barrier();
    slot = slot == T_RING - 1 ? 0 : slot + 1;
    pslot = pslot == T_RING - 1 ? 0 : pslot + 1;
  }
  if (wr == 0) __builtin_amdgcn_s_barrier();

  float* P = a.P + (long)sp * a.N * a.K;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int n = n0 + wr * 128 + i * 16 + fr;
    if (n >= a.N) continue;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int k = k0 + wc * 64 + j * 16 + 4 * fg;
      if (k < a.K) *reinterpret_cast<f32x4*>(P + (long)n * a.K + k) = acc[i][j];
    }
  }
}

}  // namespace

namespace {
// Tile selection (immutable): the 256x256 8-wave kernels run dense bf16 problems with enough
// work (NT: >= 256 tiles and K >= 384, i.e. every 728 / 1024 / 1536-channel layer at
// training batch sizes; TN: N, K >= 256); everything else runs the 128x128 kernels.  The
// `tile` argument of the entry points (0 auto, 1 = 128x128, 2 = 256x256) overrides the choice
// so tests can pin each kernel at small sizes.
// 256x256 weight-gradient workgroups (splits x tiles): about half the CUs.  The engine runs the
// weight gradients on a side stream beside the main stream's dgrad GEMMs and depthwise backward;
// one 160 KB-LDS workgroup on every CU left those no room, half the CUs (and half the split-K
// slabs) measured 1.0-1.8 % faster per step for targets 64-192 (profiles/r02_tn_target_sweep.txt).
constexpr int TN_TARGET_WGS_DEFAULT = 128;
bool tn_xcd_splits() {   // XCP_TN_XCD_SPLITS=1 (A/B; measured -0.3 % in the step, off)
  static const bool v = [] {
    const char* e = getenv("XCP_TN_XCD_SPLITS");
    return e && e[0] == '1';
  }();
  return v;
}
// The weight-gradient kernel with one 32-MFMA phase per step and the fill 4 steps ahead (gemm_tn256q_kernel):
// 9-13 % faster alone at every step shape, the partial slabs bitwise equal (profiles/r06_tn_loop_ab.txt).
// XCP_TN_LOOP=1: gemm_tn256_kernel's two 16-MFMA phases (read per call; A/B)
bool tn_loop2() {
  const char* e = getenv("XCP_TN_LOOP");
  return !(e && e[0] == '1');
}
// XCP_TN_XCD_ALIGN=1: whole splits per XCD for outputs of at most 32 tiles (read per call; A/B)
bool tn_xcd_align() {
  const char* e = getenv("XCP_TN_XCD_ALIGN");
  return e && e[0] == '1';
}
int tn_target_wgs() {   // XCP_TN_TARGET_WGS=<n> overrides the default (A/B of the side-stream share)
  static const int v = [] {
    const char* e = getenv("XCP_TN_TARGET_WGS");
    const int n = e ? atoi(e) : 0;
    return n > 0 ? n : TN_TARGET_WGS_DEFAULT;
  }();
  return v;
}

int gpu_cus() {   // compute units of the current device (256 on MI355X)
  static const int cus = [] {
    int d = 0, n = 0;
    if (hipGetDevice(&d) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, d) != hipSuccess)
      n = 0;
    return n > 0 ? n : 256;
  }();
  return cus;
}

int nt_big_min_k() {   // XCP_NT_BIG_MINK=<k>: smallest K the automatic choice gives the 256x256 kernel (A/B)
  static const int v = [] {
    const char* e = getenv("XCP_NT_BIG_MINK");
    const int k = e ? atoi(e) : 0;
    return k > 0 ? k : 384;
  }();
  return v;
}

// Outputs at least 256 wide also take the 256x256 kernel from K = 128 (entry-flow forward GEMMs,
// tools/kbench.py entrygemm, profiles/r03_entrygemm.txt: 1,401,856 x 256 x 128 / 256 297 -> 241 /
// 400 -> 318 us, 350,464 x 736 x 256 303 -> 219 us); 128-wide outputs stay on the 128x128 kernel
// (5,531,904 x 128 x 64 / 128: 459 / 567 us there against 552 / 680 on the 256x256 one).
// XCP_NT_BIG_N256=0 restores the K >= 384 rule alone (A/B).
bool nt_big_n256() {
  static const bool v = [] {
    const char* e = getenv("XCP_NT_BIG_N256");
    return !(e && e[0] == '0');
  }();
  return v;
}

// XCP_NT_SPARSE=0: no sparse last round (every row on the persistent kernel; read per call; A/B)
bool nt_sparse() {
  const char* e = getenv("XCP_NT_SPARSE");
  return !(e && e[0] == '0');
}

bool nt_big(int dtype, int gmode, int M, int N, int K, int tile) {
  if (dtype != XCP_BF16 || gmode != 0 || tile == 1) return false;
  if (tile == 2 || tile == 3) return true;
  if (xcp_cdiv(M, 256) * xcp_cdiv(N, 256) < 256) return false;
  return K >= nt_big_min_k() || (nt_big_n256() && N >= 256 && K >= 128);
}

bool tn_big(int dtype, int gmode, int N, int K, int tile) {
  // (narrower outputs stream faster through the 128-tile kernel: 0.57 vs 0.95 ms at 5.5M x 128 x 128)
  if (dtype != XCP_BF16 || gmode != 0 || tile == 1) return false;
  return tile == 2 || (N >= 256 && K >= 256);
}
}  // namespace

// XCP_NT_LOOP=4: the persistent NT kernel with four MFMA phases per K-tile (gemm_nt256p_kernel) instead of
// two (gemm_nt256q_kernel; A/B, read per call)
bool nt_loop2() {
  const char* e = getenv("XCP_NT_LOOP");
  return e && e[0] == '2';
}
bool nt_8w() {   // XCP_NT_8W=1: gemm_nt8w_kernel for the persistent calls from K = 128 (read per call; A/B)
  const char* e = getenv("XCP_NT_8W");
  return e && e[0] == '1';
}
bool nt_4w() {   // XCP_NT_4W=1 / 2: gemm_nt4w_kernel (one wave per SIMD) for the persistent calls from K = 128 (read per call; A/B)
  const char* e = getenv("XCP_NT_4W");
  return e && (e[0] == '1' || e[0] == '2');
}
bool nt_4w_ilv() {   // XCP_NT_4W=2: its steps fenced per 8-MFMA group
  const char* e = getenv("XCP_NT_4W");
  return e && e[0] == '2';
}
bool nt_pf2() {   // XCP_NT_PF2=1: gemm_nt256p_kernel's two-K-tile prefetch at tile boundaries (read per call; A/B)
  const char* e = getenv("XCP_NT_PF2");
  return e && e[0] == '1';
}
// The 256p kernel's last K-tile multiplies only its first 32-deep half when the rest of it is past K (the
// 728-channel flow at its 736 pitch: K = 728 / 736, 24 / 32 of the last 64): 32 of the tile's 768 MFMAs
// per wave skipped, C and the statistics bitwise equal (the skipped products are +0).  XCP_NT_KHALF=0:
// every K-tile whole (read per call; A/B)
bool nt_khalf() {
  const char* e = getenv("XCP_NT_KHALF");
  return !(e && e[0] == '0');
}
bool nt_half() {   // XCP_NT_HALF=1 (read per call; A/B)
  const char* e = getenv("XCP_NT_HALF");
  return e && e[0] == '1';
}

// XCP_NT_DYNQ=0: the persistent NT kernel walks its static tile list (A/B; read per call)
bool nt_dynq() {
  const char* e = getenv("XCP_NT_DYNQ");
  return !(e && e[0] == '0');
}
bool nt_sparse_dgrad() {   // XCP_NT_SPARSE_DGRAD=1 (A/B; read per call)
  const char* e = getenv("XCP_NT_SPARSE_DGRAD");
  return e && e[0] == '1';
}
// A tile-queue counter is keyed by the (device, stream) of the launch, and each launch relies on being
// its counter's only user between its first fetch and its last (which resets it).  Launches on one
// stream are ordered, so eager use is safe.  A graph node would keep the capture stream's counter
// whatever stream the graph is replayed on (and two replays could overlap), so calls under stream
// capture take the static tile walk instead.
bool stream_capturing(hipStream_t st) {
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  return hipStreamIsCapturing(st, &cs) == hipSuccess && cs != hipStreamCaptureStatusNone;
}
// tile-queue slot + 1 of (device, stream) for gemm_nt256p_kernel (0: static walk, past 64 streams)
int nt_tq_slot(hipStream_t st) {
  if (!nt_dynq()) return 0;
  static std::mutex mu;
  static std::vector<std::pair<int, hipStream_t>> slots;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 0;
  std::lock_guard<std::mutex> lk(mu);
  for (size_t i = 0; i < slots.size(); ++i)
    if (slots[i].first == dev && slots[i].second == st) return (int)i + 1;
  if (slots.size() >= 64) return 0;
  slots.emplace_back(dev, st);
  return (int)slots.size();
}

extern "C" {

// C[M,N] = A[M,K] . B[N,K]^T ; see include/xcp.h
int xcp_gemm_nt(int dtype, const void* A, long lda, const void* B, long ldb, void* C, long ldc, int M, int N, int K,
                float* stats, int gmode, int gH, int gW, int gOH, int gOW, int gS, int gC, int tile, hipStream_t stream) {
  if (M <= 0 || N <= 0 || K <= 0) return XCP_OK;
  if ((K % 8) || (N % 8) || (lda % 8) || (ldb % 8) || (ldc % 8)) return XCP_EINVAL;
  if (gmode < 0 || gmode > 3 || (gmode >= 2 && (gC % 8 || gC * 9 != K))) return XCP_EINVAL;
  if (tile < 0 || tile > 4) return XCP_EINVAL;
  NTArgs a{A, lda, B, ldb, C, ldc, M, N, K, stats, Gather{gmode, gH, gW, gOH, gOW, gS > 0 ? gS : 1, gC}};
  a.khalf = nt_khalf() ? 1 : 0;
  if (nt_big(dtype, gmode, M, N, K, tile)) {
    // automatic choice (tile 0): the persistent kernel; tile 4: the automatic choice with the
    // one-shot kernel (A/B)
    const bool persist = tile == 3 || tile == 0;
    // One 256x256 tile per CU per round.  When the last round would be less than 3/4 full
    // (1,083 tiles = 4.23 rounds in the middle flow), its rows go to the 128x128 kernel
    // instead: four times as many, smaller tiles, one launch after the full rounds
    // (tile 0 / 4 only; tile 2 pins the one-shot 256 kernel for every row, tile 3 the persistent one).
    const int gridN = xcp_cdiv(N, 256), gridM = xcp_cdiv(M, 256), tiles = gridM * gridN;
    const int cus = gpu_cus();
    int mb = gridM;
    // (calls that take the tile queue keep every row on the persistent kernel: the queue spreads the last
    // round's tiles over whichever workgroups finish first; +0.2 % in the step, profiles/r05_nt_dynq_ab.txt;
    // XCP_NT_SPARSE_DGRAD=1 moves their sparse last round to the 128x128 kernel as before)
    const bool queued = tile == 0 && K >= 128 && !stats && nt_dynq();
    const bool partial = tiles > cus && tiles % cus != 0 && (tiles % cus) * 4 < cus * 3;   // last round < 3/4 full
    // XCP_NT_HALF=1: the last round's tiles as half tiles walked FIRST by the persistent kernel (every row on it;
    // the half-tile workgroups run half a tile out of step with the rest, so the rounds' epilogue store bursts
    // are split in two)
    const bool halves = tile == 0 && persist && partial && K > 64 && nt_half() && !nt_loop2();
    if ((tile == 0 || tile == 4) && !halves && nt_sparse() && (!queued || nt_sparse_dgrad()) && partial)
      mb = (tiles / cus) * cus / gridN;
    NTArgs big = a;
    big.M = min(M, mb * 256);
    if (halves) big.nsplit = tiles % cus;
    const bool buf = ((long)(big.M - 1) * lda + K) * 2 <= BUF_LIMIT && ((long)(N - 1) * ldb + K) * 2 <= BUF_LIMIT;
    const bool cbuf = ((long)(big.M - 1) * ldc + N) * 2 <= BUF_LIMIT && (!stats || (long)xcp_cdiv(M, 128) * 2 * N * 4 <= BUF_LIMIT);
    if (persist && buf && cbuf) {   // persistent: one workgroup per CU walks the tiles
      const int grid = min(mb * gridN, cus);
      // the tile queue for the calls without BN statistics: the backward's input gradients, which run beside
      // the side stream's weight gradients (the forward's launches have the GPU to themselves and keep
      // the static XCD-ordered walk: with the queue they measured 1 % slower); K >= 128: the counter's
      // fetch retires within two K-tiles
      big.tqs = K >= 128 && !stats && !stream_capturing(stream) ? nt_tq_slot(stream) : 0;
      if (K > 64 && nt_loop2()) {   // two MFMA phases per K-tile, fill 1.5 K-tiles ahead
        if (stats)
          hipLaunchKernelGGL(gemm_nt256q_kernel<true>, dim3(grid), dim3(512), 0, stream, big);
        else
          hipLaunchKernelGGL(gemm_nt256q_kernel<false>, dim3(grid), dim3(512), 0, stream, big);
      } else if (halves) {
        if (stats)
          hipLaunchKernelGGL((gemm_nt256p_kernel<true, true, false>), dim3(grid), dim3(512), 0, stream, big);
        else
          hipLaunchKernelGGL((gemm_nt256p_kernel<false, true, false>), dim3(grid), dim3(512), 0, stream, big);
      } else if (nt_8w() && K >= 128) {
        if (stats)
          hipLaunchKernelGGL(gemm_nt8w_kernel<true>, dim3(grid), dim3(512), 0, stream, big);
        else
          hipLaunchKernelGGL(gemm_nt8w_kernel<false>, dim3(grid), dim3(512), 0, stream, big);
      } else if (nt_4w() && K >= 128) {
        const bool ilv = nt_4w_ilv();
        if (stats && ilv)
          hipLaunchKernelGGL((gemm_nt4w_kernel<true, true>), dim3(grid), dim3(256), 0, stream, big);
        else if (stats)
          hipLaunchKernelGGL((gemm_nt4w_kernel<true, false>), dim3(grid), dim3(256), 0, stream, big);
        else if (ilv)
          hipLaunchKernelGGL((gemm_nt4w_kernel<false, true>), dim3(grid), dim3(256), 0, stream, big);
        else
          hipLaunchKernelGGL((gemm_nt4w_kernel<false, false>), dim3(grid), dim3(256), 0, stream, big);
      } else if (nt_pf2()) {
        if (stats)
          hipLaunchKernelGGL((gemm_nt256p_kernel<true, false, true>), dim3(grid), dim3(512), 0, stream, big);
        else
          hipLaunchKernelGGL((gemm_nt256p_kernel<false, false, true>), dim3(grid), dim3(512), 0, stream, big);
      } else if (stats)
        hipLaunchKernelGGL((gemm_nt256p_kernel<true, false, false>), dim3(grid), dim3(512), 0, stream, big);
      else
        hipLaunchKernelGGL((gemm_nt256p_kernel<false, false, false>), dim3(grid), dim3(512), 0, stream, big);
    } else if (buf)
      hipLaunchKernelGGL(gemm_nt256k64_kernel<true>, dim3(mb * gridN), dim3(512), 0, stream, big);
    else
      hipLaunchKernelGGL(gemm_nt256k64_kernel<false>, dim3(mb * gridN), dim3(512), 0, stream, big);
    if (big.M < M) {
      NTArgs rest = a;
      rest.M = M - big.M;
      rest.A = reinterpret_cast<const bf16*>(A) + (long)big.M * lda;
      rest.C = reinterpret_cast<bf16*>(C) + (long)big.M * ldc;
      if (stats) rest.stats = stats + (long)(big.M / 128) * 2 * N;
      hipLaunchKernelGGL((gemm_nt_kernel<bf16, 0, 2, 2>), dim3(xcp_cdiv(rest.M, 128) * xcp_cdiv(N, NBN)), dim3(256), 0,
                         stream, rest);
    }
    return (int)hipGetLastError();
  }
  const int grid = xcp_cdiv(M, 128) * xcp_cdiv(N, NBN);
#define XCP_NT_LAUNCH(TT)                                                                                       \
  switch (gmode) {                                                                                              \
    case 0: hipLaunchKernelGGL((gemm_nt_kernel<TT, 0, 2, 2>), dim3(grid), dim3(256), 0, stream, a); break;     \
    case 1: hipLaunchKernelGGL((gemm_nt_kernel<TT, 1, 2, 2>), dim3(grid), dim3(256), 0, stream, a); break;     \
    case 2: hipLaunchKernelGGL((gemm_nt_kernel<TT, 2, 2, 2>), dim3(grid), dim3(256), 0, stream, a); break;     \
    default: hipLaunchKernelGGL((gemm_nt_kernel<TT, 3, 2, 2>), dim3(grid), dim3(256), 0, stream, a); break;    \
  }
  if (dtype == XCP_BF16) {
    XCP_NT_LAUNCH(bf16)
  } else if (dtype == XCP_F32) {
    XCP_NT_LAUNCH(float)
  } else {
    return XCP_EUNSUPPORTED;
  }
#undef XCP_NT_LAUNCH
  return (int)hipGetLastError();
}

// rows of the stats partial array gemm_nt writes ([rows][2][N]): one per 128 output rows for
// both tile sizes (the 256-row kernel writes one row per 128-row half)
int xcp_gemm_nt_stat_rows(int M) { return xcp_cdiv(M, 128); }

// Rows per split for xcp_gemm_tn (S = ceil(M / rows)): about one workgroup per CU for
// the 256x256 kernel (each split's partial slab costs 4*N*K bytes of writes and
// reads), ~1024 workgroups of the 128x128 kernel otherwise.
int xcp_gemm_tn_rows_per_split(int dtype, int gmode, int M, int N, int K, int tile) {
  if (M <= 0) return 64;
  const bool big = tn_big(dtype, gmode, N, K, tile);
  const int tsz = big ? 256 : 128, align = big ? 64 : 32;
  const int tiles = xcp_cdiv(N, tsz) * xcp_cdiv(K, tsz);
  const int target = big ? tn_target_wgs() : 1024, min_rows = big ? 512 : 256;
  int S = target / (tiles > 0 ? tiles : 1);
  S = S < 1 ? 1 : S;
  // XCP_TN_XCD_SPLITS=1: for few output tiles a multiple of 8 splits, so that with the kernel's
  // XCD remap every XCD holds whole splits and a split's row panels are shared by all of its tiles
  // in one L2 (9 tiles x 14 splits = 126 workgroups put most splits across two XCDs).  Measured in
  // the step: 399.6-400.4 vs 400.7-401.3 clips/s with the plain count (profiles/r03_ab3.txt): off.
  if (big && tiles <= 16 && S >= 4 && tn_xcd_splits()) S = (S + 4) / 8 * 8;
  const int smax = xcp_cdiv(M, min_rows);
  S = S < smax ? S : smax;
  int rps = xcp_cdiv(M, S);
  rps = xcp_cdiv(rps, align) * align;
  return rps;
}

// P[s][N][K] partial weight gradients; S splits of rows_per_split rows each.
int xcp_gemm_tn(int dtype, const void* G, long ldg, const void* X, long ldx, float* P, int M, int N, int K, int S,
                int rows_per_split, int gmode, int gH, int gW, int gOH, int gOW, int gS, int gC, int tile,
                hipStream_t stream) {
  if (N <= 0 || K <= 0 || S <= 0) return XCP_OK;
  if ((K % 8) || (N % 8) || (ldg % 8) || (ldx % 8)) return XCP_EINVAL;
  if (gmode < 0 || gmode > 2 || (gmode == 2 && (gC % 8 || gC * 9 != K))) return XCP_EINVAL;
  if (tile < 0 || tile > 2) return XCP_EINVAL;
  TNArgs a{G, ldg, X, ldx, P, M, N, K, S, rows_per_split, Gather{gmode, gH, gW, gOH, gOW, gS > 0 ? gS : 1, gC}};
  if (tn_big(dtype, gmode, N, K, tile)) {
    if (rows_per_split % 32) return XCP_EINVAL;
    const int tiles = xcp_cdiv(N, 256) * xcp_cdiv(K, 256);
    a.xalign = tiles <= 32 && S >= 2 && tn_xcd_align();
    const dim3 grid(a.xalign ? 8 * xcp_cdiv(S, 8) * tiles : tiles * S);
    const bool buf = ((long)(M - 1) * ldg + N) * 2 <= BUF_LIMIT && ((long)(M - 1) * ldx + K) * 2 <= BUF_LIMIT;
    if (tn_loop2()) {
      if (buf)
        hipLaunchKernelGGL(gemm_tn256q_kernel<true>, grid, dim3(512), 0, stream, a);
      else
        hipLaunchKernelGGL(gemm_tn256q_kernel<false>, grid, dim3(512), 0, stream, a);
    } else if (buf)
      hipLaunchKernelGGL(gemm_tn256_kernel<true>, grid, dim3(512), 0, stream, a);
    else
      hipLaunchKernelGGL(gemm_tn256_kernel<false>, grid, dim3(512), 0, stream, a);
    return (int)hipGetLastError();
  }
  const int grid = xcp_cdiv(N, 128) * xcp_cdiv(K, 128) * S;
#define XCP_TN_LAUNCH(TT)                                                                                      \
  switch (gmode) {                                                                                             \
    case 0: hipLaunchKernelGGL((gemm_tn_kernel<TT, 0>), dim3(grid), dim3(NT), 0, stream, a); break;          \
    case 1: hipLaunchKernelGGL((gemm_tn_kernel<TT, 1>), dim3(grid), dim3(NT), 0, stream, a); break;          \
    default: hipLaunchKernelGGL((gemm_tn_kernel<TT, 2>), dim3(grid), dim3(NT), 0, stream, a); break;         \
  }
  if (dtype == XCP_BF16) {
    XCP_TN_LAUNCH(bf16)
  } else if (dtype == XCP_F32) {
    XCP_TN_LAUNCH(float)
  } else {
    return XCP_EUNSUPPORTED;
  }
#undef XCP_TN_LAUNCH
  return (int)hipGetLastError();
}

}  // extern "C"
