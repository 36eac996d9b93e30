// BatchNorm2d (train-mode batch statistics / eval-mode running statistics),
// the block tails (MaxPool 3x3 s2 p1 + residual add), the final BN+ReLU+global
// average pool, and their backward passes.  NHWC rows of C channels.
//
// Reference ops: nn.BatchNorm2d (Xception.py:56,67,73,78,119,123,143,147),
// nn.MaxPool2d(3, strides, 1) (:86), residual `x += skip` (:98),
// F.adaptive_avg_pool2d (:197), ReLU (:60,:83,:170,:174,:191,:195).
//
// Statistics are reduced deterministically: producers write fp32 per-tile
// partial rows [R][2][C]; the finalize kernels fold them in fp64.  Normalisation uses the biased batch variance,
// running_var is updated with the unbiased one (momentum 0.1), as PyTorch does.
#include "common.h"

namespace {

// ---------------------------------------------------------------- column reduce
// out[g][l] = sum_{s in group g} in[s][l]   (in: fp32 [S][ld], l < L <= ld; out: fp32 [G][L];
// ACC: out +=).  Lane = VEC consecutive columns, wave w of 4 takes slabs w, w+4, ... of its group with four
// loads in flight (the adds stay in slab order), the block folds the 4 waves in fp64.
// The summation order depends only on (S, L, G), so the result is deterministic.
template <bool ACC, int VEC>
__global__ __launch_bounds__(256) void colreduce_kernel(const float* __restrict__ in, int S, long L, long ld,
                                                        float* __restrict__ out, int G) {
  __shared__ double red[4][64 * VEC];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const long col = ((long)blockIdx.x * 64 + lane) * VEC;
  const int g = blockIdx.y;
  const int spg = (S + G - 1) / G;
  const int s0 = g * spg, s1 = min(S, s0 + spg);
  double acc[VEC];
#pragma unroll
  for (int j = 0; j < VEC; ++j) acc[j] = 0.0;
  if (col < L) {
    const float* p = in + col;
    int s = s0 + w;
    for (; s + 12 < s1; s += 16) {
      float v[4][VEC];
#pragma unroll
      for (int u = 0; u < 4; ++u) VecIO<float, VEC>::load(p + (long)(s + 4 * u) * ld, v[u]);
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int j = 0; j < VEC; ++j) acc[j] += (double)v[u][j];
    }
    for (; s < s1; s += 4) {
      float v[VEC];
      VecIO<float, VEC>::load(p + (long)s * ld, v);
#pragma unroll
      for (int j = 0; j < VEC; ++j) acc[j] += (double)v[j];
    }
  }
#pragma unroll
  for (int j = 0; j < VEC; ++j) red[w][lane * VEC + j] = acc[j];
  __syncthreads();
  if (w == 0 && col < L) {
    float v[VEC], o[VEC];
#pragma unroll
    for (int j = 0; j < VEC; ++j) {
      const int i = lane * VEC + j;
      v[j] = (float)(red[0][i] + red[1][i] + red[2][i] + red[3][i]);
    }
    float* q = out + (long)g * L + col;
    if (ACC) {
      VecIO<float, VEC>::load(q, o);
#pragma unroll
      for (int j = 0; j < VEC; ++j) v[j] += o[j];
    }
    VecIO<float, VEC>::store(q, v);
  }
}

// Several independent column reductions in one launch (the weight-gradient slab reductions of
// one backbone block: its pointwise split-K slabs and depthwise partials), jobs passed by value
// in the kernel arguments.  Each job runs colreduce_kernel's arithmetic (VEC = 4) on its own
// blocks, so every output is bitwise what the single-job launch gives.
constexpr int CR_MAXJ = 16;
struct CRJob {
  const float* in;
  float* out;
  long L, ld;
  int S, G, acc, blk0, nbx;
};
struct CRMulti {
  CRJob j[CR_MAXJ];
  int njobs;
};

__global__ __launch_bounds__(256) void colreduce_multi_kernel(CRMulti m) {
  __shared__ double red[4][64 * 4];
  int k = 0;
#pragma unroll 1
  while (k + 1 < m.njobs && (int)blockIdx.x >= m.j[k + 1].blk0) ++k;
  const CRJob jb = m.j[k];
  const int local = blockIdx.x - jb.blk0;
  const int g = local / jb.nbx, bx = local - g * jb.nbx;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const long col = ((long)bx * 64 + lane) * 4;
  const int spg = (jb.S + jb.G - 1) / jb.G;
  const int s0 = g * spg, s1 = min(jb.S, s0 + spg);
  double acc[4] = {0.0, 0.0, 0.0, 0.0};
  if (col < jb.L) {
    const float* p = jb.in + col;
    int s = s0 + w;
    for (; s + 12 < s1; s += 16) {
      float v[4][4];
#pragma unroll
      for (int u = 0; u < 4; ++u) VecIO<float, 4>::load(p + (long)(s + 4 * u) * jb.ld, v[u]);
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int q = 0; q < 4; ++q) acc[q] += (double)v[u][q];
    }
    for (; s < s1; s += 4) {
      float v[4];
      VecIO<float, 4>::load(p + (long)s * jb.ld, v);
#pragma unroll
      for (int q = 0; q < 4; ++q) acc[q] += (double)v[q];
    }
  }
#pragma unroll
  for (int q = 0; q < 4; ++q) red[w][lane * 4 + q] = acc[q];
  __syncthreads();
  if (w == 0 && col < jb.L) {
    float v[4], o[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int i = lane * 4 + q;
      v[q] = (float)(red[0][i] + red[1][i] + red[2][i] + red[3][i]);
    }
    float* dst = jb.out + (long)g * jb.L + col;
    if (jb.acc) {
      VecIO<float, 4>::load(dst, o);
#pragma unroll
      for (int q = 0; q < 4; ++q) v[q] += o[q];
    }
    VecIO<float, 4>::store(dst, v);
  }
}

// ---------------------------------------------------------------- per-channel reductions
// Generic channel-reduction skeleton: block = nch channel chunks x P row chunks;
// thread (lcv, slot) accumulates CPT channels over rows slot, slot+SPB, ... of its
// row chunk; the block folds the slots in LDS and writes partial[pchunk][2][C].
struct ChanRed {
  int C, CV, CVB, SPB, nch;
  long rows, rows_per_chunk;
};

ChanRed make_chanred(long rows, int C, int CPT, int target_blocks) {
  ChanRed r;
  r.C = C;
  r.CV = C / CPT;
  r.nch = (r.CV + 63) / 64;
  r.CVB = (r.CV + r.nch - 1) / r.nch;
  r.SPB = 256 / r.CVB;
  long P = target_blocks / r.nch;
  if (P < 1) P = 1;
  const long maxP = (rows + 4L * r.SPB - 1) / (4L * r.SPB);
  if (P > maxP) P = maxP;
  if (P < 1) P = 1;
  r.rows = rows;
  r.rows_per_chunk = (rows + P - 1) / P;
  return r;
}
long chanred_P(const ChanRed& r) { return (r.rows + r.rows_per_chunk - 1) / r.rows_per_chunk; }

template <int CPT>
XCP_DEV void chanred_finish(const ChanRed& r, float (*acc)[CPT], float* part, int cchunk, int pchunk, int lcv, int slot) {
  extern __shared__ __attribute__((aligned(16))) float red[];   // [SPB][2][CVB*CPT]
  const int L = r.CVB * CPT;
  if (slot < r.SPB) {
#pragma unroll
    for (int j = 0; j < CPT; ++j) {
      red[(slot * 2 + 0) * L + lcv * CPT + j] = acc[0][j];
      red[(slot * 2 + 1) * L + lcv * CPT + j] = acc[1][j];
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 2 * L; i += 256) {
    const int k = i / L, cl = i % L;
    float s = 0.f;
    for (int q = 0; q < r.SPB; ++q) s += red[(q * 2 + k) * L + cl];
    const int c = cchunk * L + cl;
    if (c < r.C) part[((long)pchunk * 2 + k) * r.C + c] = s;
  }
}

// Source of the MaxPool2d(3, 2, 1) (Xception.py:86) gradient: the pooled gradient dOut and the
// forward's argmax taps (amax, one byte per element, read 8 at a time).
struct PoolSrc {
  const void* dOut;
  const unsigned char* amax;
  int H, W, OH, OW;
};

// raw storage of CPT elements of T (one vector load)
template <typename T, int CPT> struct RawVec;
template <> struct RawVec<bf16, 8> { typedef uint4 type; };
template <> struct RawVec<bf16, 4> { typedef uint2 type; };
template <> struct RawVec<bf16, 2> { typedef unsigned type; };
struct U4x2 { uint4 a, b; };
template <> struct RawVec<float, 8> { typedef U4x2 type; };
template <> struct RawVec<float, 4> { typedef uint4 type; };
template <> struct RawVec<float, 2> { typedef uint2 type; };
template <> struct RawVec<float, 1> { typedef unsigned type; };

// MODE 0: (x, x^2) of rows of X.  MODE 1: (dz, dz*yhat), yhat = (y-mean)*invstd.
// MODE 2: MODE 1 with dz masked by the ReLU that followed the BN (y*ms+mt > 0), i.e. the
// gradient w.r.t. relu(bn(y)) given; the mask is recomputed from y, never read.
template <typename T, int MODE, int CPT>
__global__ __launch_bounds__(256) void chanred_kernel(ChanRed r, const void* Av, const void* Bv, const float* mean,
                                                      const float* invstd, const float* ms, const float* mt,
                                                      float* part) {
  const int cchunk = blockIdx.x % r.nch, pchunk = blockIdx.x / r.nch;
  const int lcv = threadIdx.x % r.CVB, slot = threadIdx.x / r.CVB;
  const int cv = cchunk * r.CVB + lcv;
  const int c0 = cv * CPT;
  const T* A = reinterpret_cast<const T*>(Av);
  const T* B = reinterpret_cast<const T*>(Bv);
  float acc[2][CPT];
#pragma unroll
  for (int j = 0; j < CPT; ++j) acc[0][j] = acc[1][j] = 0.f;
  if (slot < r.SPB && cv < r.CV) {
    float mu[CPT], is[CPT], sm[CPT], tm[CPT];
    if constexpr (MODE >= 1) {
      VecIO<float, CPT>::load(mean + c0, mu);
      VecIO<float, CPT>::load(invstd + c0, is);
    }
    if constexpr (MODE == 2) {
      VecIO<float, CPT>::load(ms + c0, sm);
      VecIO<float, CPT>::load(mt + c0, tm);
    }
    const long rb = (long)pchunk * r.rows_per_chunk, re = min(r.rows, rb + r.rows_per_chunk);
    // rows in groups of CR_U: every raw load of a group is issued before the first is used
    // (clamped row, masked past the chunk), so a thread waits one memory round trip per CR_U rows
    // instead of one per row (middle flow: 36 rows per thread, 36 -> 5 round trips)
    constexpr int CR_U = 8;
    constexpr int NB = MODE == 0 ? 1 : 2;
    typedef typename RawVec<T, CPT>::type RV;
    // (32-bit element offsets: the launcher checks rows * C < 2^31; a 64-bit product per load was three
    // quarter-rate multiplies)
    const unsigned last = (unsigned)(re - 1) * (unsigned)r.C + (unsigned)c0, ustep = (unsigned)r.SPB * (unsigned)r.C;
    for (long p0 = rb + slot; p0 < re; p0 += (long)CR_U * r.SPB) {
      RV raw[NB][CR_U];
      const unsigned o0 = (unsigned)p0 * (unsigned)r.C + (unsigned)c0;
#pragma unroll
      for (int u = 0; u < CR_U; ++u) {
        const unsigned o = min(o0 + (unsigned)u * ustep, last);
        raw[0][u] = *reinterpret_cast<const RV*>(A + o);
        if constexpr (MODE >= 1) raw[NB - 1][u] = *reinterpret_cast<const RV*>(B + o);
      }
      __builtin_amdgcn_sched_barrier(0);   // (the scheduler would sink each load to its use)
#pragma unroll
      for (int u = 0; u < CR_U; ++u) {
        const bool ok = p0 + (long)u * r.SPB < re;   // (a select, not a branch: the loads stay ahead)
        float a[CPT];
        VecIO<T, CPT>::load(reinterpret_cast<const T*>(&raw[0][u]), a);
#pragma unroll
        for (int j = 0; j < CPT; ++j) a[j] = ok ? a[j] : 0.f;
        if constexpr (MODE == 0) {
#pragma unroll
          for (int j = 0; j < CPT; ++j) {
            acc[0][j] += a[j];
            acc[1][j] = fmaf(a[j], a[j], acc[1][j]);
          }
        } else {
          float b[CPT];
          VecIO<T, CPT>::load(reinterpret_cast<const T*>(&raw[NB - 1][u]), b);
          if constexpr (MODE == 2) {
#pragma unroll
            for (int j = 0; j < CPT; ++j) a[j] = fmaf(b[j], sm[j], tm[j]) > 0.f ? a[j] : 0.f;
          }
#pragma unroll
          for (int j = 0; j < CPT; ++j) {
            acc[0][j] += a[j];
            acc[1][j] = fmaf(a[j], (b[j] - mu[j]) * is[j], acc[1][j]);
          }
        }
      }
    }
  }
  chanred_finish<CPT>(r, acc, part, cchunk, pchunk, lcv, slot);
}

// ---------------------------------------------------------------- finalize
// C channels of a tensor whose channel pitch is CP >= C: partial rows have CP entries per
// statistic and the per-channel outputs get CP entries, zero for the padding channels (so a
// BN-apply over the padded pitch leaves them zero).
__global__ void bn_finalize_kernel(const double* __restrict__ part2, int G, int C, int CP, double count,
                                   const float* gamma, const float* beta, float* rmean, float* rvar, float momentum,
                                   float eps, int train, float* mean_o, float* invstd_o, float* scale_o,
                                   float* shift_o) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= CP) return;
  if (c >= C) {
    mean_o[c] = invstd_o[c] = scale_o[c] = shift_o[c] = 0.f;
    return;
  }
  double mean, var;
  if (train) {
    double s = 0.0, q = 0.0;
    for (int g = 0; g < G; ++g) {
      s += part2[((long)g * 2 + 0) * CP + c];
      q += part2[((long)g * 2 + 1) * CP + c];
    }
    mean = s / count;
    var = q / count - mean * mean;
    if (var < 0.0) var = 0.0;
    if (rmean) {
      const double unb = count > 1.0 ? var * count / (count - 1.0) : var;
      rmean[c] = (float)((1.0 - momentum) * rmean[c] + momentum * mean);
      rvar[c] = (float)((1.0 - momentum) * rvar[c] + momentum * unb);
    }
  } else {
    mean = rmean[c];
    var = rvar[c];
  }
  const float is = (float)(1.0 / sqrt(var + (double)eps));
  const float sc = gamma[c] * is;
  mean_o[c] = (float)mean;
  invstd_o[c] = is;
  scale_o[c] = sc;
  shift_o[c] = beta[c] - (float)mean * sc;
}

// Fused reduction + finalize straight from the fp32 partial rows part[R][2][C] (the GEMM
// epilogue's / the fused depthwise backward's per-chunk sums): one 1024-thread workgroup
// per 32 channels; lane l of wave w sums statistic l>>5 of channel l&31 over rows w, w+16, ... in fp64 (four independent accumulators, so
// many loads stay in flight), the 16 waves fold in LDS, and 32 threads finalize.
// FIN_WAVES_NARROW (xcp_bn_bwd_finalize_part flag XCP_FIN_NARROW): 4 waves -- one per SIMD, 58 VGPRs each -- fit
// beside a kernel that holds every CU (the stem conv2 weight gradient: 2 waves x 169 VGPRs per SIMD), where the
// 16-wave workgroup (4 per SIMD) waited for it to finish (144 us per step)
constexpr int FIN_CH = 32, FIN_WAVES = 16, FIN_WAVES_NARROW = 4;

template <int NW>
XCP_DEV void fin_reduce(const float* __restrict__ part, int R, int C, int CP, int c0, double (*red)[64], double& s0,
                        double& s1) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c = c0 + (lane & 31), stat = lane >> 5;
  // rows w, w + 16, ... in chunks of FIN_U: every load of a chunk is issued before the first is
  // added (clamped row, zero-selected past R), so a lane waits ceil(R / (16 FIN_U)) memory round
  // trips, not one per 4 rows (723 partial rows of the middle flow: one; the same summation order
  // as smaller chunks, so the same bits)
  // (the row offsets are wave-uniform, so they are formed on the scalar unit: the 64-bit product per
  // load in vector registers was three quarter-rate multiplies, 144 in the loop)
  constexpr int FIN_U = 48;
  double a = 0.0;
  if (c < C) {
    const float* col = part + (long)stat * CP + c;
    const int ws = __builtin_amdgcn_readfirstlane(w);
    for (int r0 = ws; r0 < R; r0 += FIN_U * NW) {
      float v[FIN_U];
#pragma unroll
      for (int u = 0; u < FIN_U; ++u) v[u] = col[min(r0 + u * NW, R - 1) * 2 * CP];
#pragma unroll
      for (int u = 0; u < FIN_U; ++u) a += r0 + u * NW < R ? (double)v[u] : 0.0;
    }
  }
  red[w][lane] = a;
  __syncthreads();
  s0 = s1 = 0.0;
  if (threadIdx.x < FIN_CH) {
#pragma unroll
    for (int q = 0; q < NW; ++q) {
      s0 += red[q][threadIdx.x];
      s1 += red[q][threadIdx.x + 32];
    }
  }
}

__global__ __launch_bounds__(64 * FIN_WAVES) void bn_finalize_part_kernel(const float* __restrict__ part, int R, int C, int CP,
                                                                double count, const float* gamma, const float* beta,
                                                                float* rmean, float* rvar, float momentum, float eps,
                                                                float* mean_o, float* invstd_o, float* scale_o,
                                                                float* shift_o) {
  __shared__ double red[FIN_WAVES][64];
  const int c0 = blockIdx.x * FIN_CH;
  double s, q;
  fin_reduce<FIN_WAVES>(part, R, C, CP, c0, red, s, q);
  const int c = c0 + threadIdx.x;
  if (threadIdx.x >= FIN_CH || c >= CP) return;
  if (c >= C) {   // padding channel
    mean_o[c] = invstd_o[c] = scale_o[c] = shift_o[c] = 0.f;
    return;
  }
  const double mean = s / count;
  double var = q / count - mean * mean;
  if (var < 0.0) var = 0.0;
  if (rmean) {
    const double unb = count > 1.0 ? var * count / (count - 1.0) : var;
    rmean[c] = (float)((1.0 - momentum) * rmean[c] + momentum * mean);
    rvar[c] = (float)((1.0 - momentum) * rvar[c] + momentum * unb);
  }
  const float is = (float)(1.0 / sqrt(var + (double)eps));
  const float sc = gamma[c] * is;
  mean_o[c] = (float)mean;
  invstd_o[c] = is;
  scale_o[c] = sc;
  shift_o[c] = beta[c] - (float)mean * sc;
}

template <int NWAVES>
__global__ __launch_bounds__(64 * NWAVES) void bn_bwd_finalize_part_kernel(const float* __restrict__ part, int R, int C,
                                                                    int CP, double count, const float* gamma,
                                                                    const float* mean, const float* invstd,
                                                                    float* alpha, float* bcoef, float* delta,
                                                                    float* dgamma, float* dbeta, int accumulate) {
  __shared__ double red[NWAVES][64];
  const int c0 = blockIdx.x * FIN_CH;
  double sdz, sdzy;
  fin_reduce<NWAVES>(part, R, C, CP, c0, red, sdz, sdzy);
  const int c = c0 + threadIdx.x;
  if (threadIdx.x >= FIN_CH || c >= CP) return;
  if (c >= C) {   // padding channel: its gradient stays zero
    alpha[c] = bcoef[c] = delta[c] = 0.f;
    return;
  }
  const double is = invstd[c], gm = gamma[c], mu = mean[c];
  const double a = gm * is;
  const double mdz = sdz / count, mdzy = sdzy / count;
  alpha[c] = (float)a;
  bcoef[c] = (float)(-a * is * mdzy);
  delta[c] = (float)(-a * mdz + a * is * mu * mdzy);
  if (dgamma) {
    dgamma[c] = accumulate ? dgamma[c] + (float)sdzy : (float)sdzy;
    dbeta[c] = accumulate ? dbeta[c] + (float)sdz : (float)sdz;
  }
}

// ---------------------------------------------------------------- elementwise
template <typename T, int CPT>
__global__ __launch_bounds__(256) void bn_act_kernel(const T* __restrict__ X, T* __restrict__ Y, const float* scale,
                                                     const float* shift, int relu, long rows, int C) {
  const int CV = C / CPT;
  const long g = (long)blockIdx.x * 256 + threadIdx.x;
  if (g >= rows * CV) return;
  const int c0 = (int)(g % CV) * CPT;
  const long p = g / CV;
  float v[CPT], s[CPT], t[CPT];
  VecIO<T, CPT>::load(X + p * C + c0, v);
  VecIO<float, CPT>::load(scale + c0, s);
  VecIO<float, CPT>::load(shift + c0, t);
#pragma unroll
  for (int j = 0; j < CPT; ++j) {
    v[j] = fmaf(v[j], s[j], t[j]);
    if (relu) v[j] = fmaxf(v[j], 0.f);
  }
  VecIO<T, CPT>::store(Y + p * C + c0, v);
}

// y[n][oh][ow] = act(x[n][oh*S][ow*S] * scale + shift): the activated input of a stride-S 1x1
// conv (Block.skip, Xception.py:55) when the consumers of the full-resolution activation
// apply the BN + ReLU on load themselves
template <typename T, int CPT>
__global__ __launch_bounds__(256) void bn_act_strided_kernel(const T* __restrict__ X, T* __restrict__ Y, const float* scale,
                                                             const float* shift, int relu, int H, int W, int OH, int OW,
                                                             int S, long rows, int C) {
  const int CV = C / CPT;
  const long g = (long)blockIdx.x * 256 + threadIdx.x;
  if (g >= rows * CV) return;
  const int c0 = (int)(g % CV) * CPT;
  const long p = g / CV;
  const long n = p / ((long)OH * OW);
  const int rem = (int)(p - n * OH * OW), oh = rem / OW, ow = rem - oh * OW;
  const long q = (n * H + (long)oh * S) * W + (long)ow * S;
  float v[CPT], s[CPT], t[CPT];
  VecIO<T, CPT>::load(X + q * C + c0, v);
  VecIO<float, CPT>::load(scale + c0, s);
  VecIO<float, CPT>::load(shift + c0, t);
#pragma unroll
  for (int j = 0; j < CPT; ++j) {
    v[j] = fmaf(v[j], s[j], t[j]);
    if (relu) v[j] = fmaxf(v[j], 0.f);
  }
  VecIO<T, CPT>::store(Y + p * C + c0, v);
}

// dy = alpha*dz + bcoef*y + delta   (dbeta = sum dz, dgamma = sum dz*yhat come from the finalize)
// A thread owns one chunk of CPT channels in RPT rows p0 + k * ceil(rows / RPT) (each k a
// contiguous stream across the grid): the 3-5 per-channel coefficient vectors are loaded once
// for RPT rows, and all 2 * RPT data loads are issued back to back (clamped rows, guarded stores).
template <typename T, int CPT, bool MASK, int RPT>
__global__ __launch_bounds__(256) void bn_bwd_apply_kernel(const T* __restrict__ dZ, const T* __restrict__ Yv, T* dY,
                                                           const float* alpha, const float* bcoef, const float* delta,
                                                           const float* ms, const float* mt, long rows, int C) {
  // 32-bit index arithmetic (the launcher checks rows * C < 2^31): a 64-bit division and 64-bit
  // address products per thread were most of its VALU
  const unsigned CV = (unsigned)C / CPT;
  const unsigned rq = (unsigned)((rows + RPT - 1) / RPT), nrows = (unsigned)rows;
  const unsigned g = blockIdx.x * 256u + threadIdx.x;
  if (g >= rq * CV) return;
  const unsigned p0 = g / CV, c0 = (g - p0 * CV) * CPT;
  const unsigned o0 = p0 * (unsigned)C + c0, ostep = rq * (unsigned)C, olast = (nrows - 1) * (unsigned)C + c0;
  float dz[RPT][CPT], y[RPT][CPT], al[CPT], bc[CPT], de[CPT];
#pragma unroll
  for (int k = 0; k < RPT; ++k) {
    const unsigned o = min(o0 + k * ostep, olast);
    VecIO<T, CPT>::load(dZ + o, dz[k]);
    VecIO<T, CPT>::load(Yv + o, y[k]);
  }
  VecIO<float, CPT>::load(alpha + c0, al);
  VecIO<float, CPT>::load(bcoef + c0, bc);
  VecIO<float, CPT>::load(delta + c0, de);
  if constexpr (MASK) {   // dZ is the gradient of relu(bn(y)): mask recomputed from y
    float sm[CPT], tm[CPT];
    VecIO<float, CPT>::load(ms + c0, sm);
    VecIO<float, CPT>::load(mt + c0, tm);
#pragma unroll
    for (int k = 0; k < RPT; ++k)
#pragma unroll
      for (int j = 0; j < CPT; ++j) dz[k][j] = fmaf(y[k][j], sm[j], tm[j]) > 0.f ? dz[k][j] : 0.f;
  }
#pragma unroll
  for (int k = 0; k < RPT; ++k) {
#pragma unroll
    for (int j = 0; j < CPT; ++j) dz[k][j] = fmaf(al[j], dz[k][j], fmaf(bc[j], y[k][j], de[j]));
    if (p0 + k * rq < nrows) VecIO<T, CPT>::store(dY + o0 + k * ostep, dz[k]);
  }
}

// dx *= (x > 0)
template <typename T, int CPT>
__global__ __launch_bounds__(256) void relu_bwd_kernel(T* dX, const T* __restrict__ Xv, long rows, int C) {
  const int CV = C / CPT;
  const long g = (long)blockIdx.x * 256 + threadIdx.x;
  if (g >= rows * CV) return;
  const int c0 = (int)(g % CV) * CPT;
  const long p = g / CV;
  float d[CPT], x[CPT];
  VecIO<T, CPT>::load(dX + p * C + c0, d);
  VecIO<T, CPT>::load(Xv + p * C + c0, x);
#pragma unroll
  for (int j = 0; j < CPT; ++j) d[j] = x[j] > 0.f ? d[j] : 0.f;
  VecIO<T, CPT>::store(dX + p * C + c0, d);
}

// Block tail: out = [maxpool3x3s2p1](y*s1+t1) + (skip_mode==0 ? inp : ys*s2+t2)
template <typename T, int CPT>
__global__ __launch_bounds__(256) void tail_fwd_kernel(const T* __restrict__ Y, const float* s1, const float* t1, int pool,
                                                       const T* __restrict__ S, const float* s2, const float* t2,
                                                       T* __restrict__ Out, unsigned char* __restrict__ amax, int N, int H,
                                                       int W, int C, int OH, int OW) {
  // 32-bit index arithmetic (the launcher checks N * H * W * C < 2^31)
  const unsigned CV = (unsigned)C / CPT;
  const unsigned g = blockIdx.x * 256u + threadIdx.x;
  if (g >= (unsigned)N * OH * OW * CV) return;
  const unsigned op = g / CV, c0 = (g - op * CV) * CPT;   // output pixel, first channel
  const unsigned t = op / OW, ow = op - t * OW;
  const unsigned n = t / OH, oh = t - n * OH;
  float sc[CPT], sh[CPT], o[CPT];
  VecIO<float, CPT>::load(s1 + c0, sc);
  VecIO<float, CPT>::load(t1 + c0, sh);
  if (pool) {
    float m[CPT];
    unsigned char am[CPT];
#pragma unroll
    for (int j = 0; j < CPT; ++j) { m[j] = -INFINITY; am[j] = 0; }
    for (int ky = 0; ky < 3; ++ky) {
      const int ih = (int)oh * 2 - 1 + ky;
      if (ih < 0 || ih >= H) continue;
      for (int kx = 0; kx < 3; ++kx) {
        const int iw = (int)ow * 2 - 1 + kx;
        if (iw < 0 || iw >= W) continue;
        float v[CPT];
        VecIO<T, CPT>::load(Y + ((n * H + ih) * W + iw) * C + c0, v);
#pragma unroll
        for (int j = 0; j < CPT; ++j) {
          const float z = fmaf(v[j], sc[j], sh[j]);
          if (z > m[j] || (z != z)) { m[j] = z; am[j] = (unsigned char)(ky * 3 + kx); }
        }
      }
    }
#pragma unroll
    for (int j = 0; j < CPT; ++j) o[j] = m[j];
    if constexpr (CPT == 8) {   // the 8 argmax bytes in one 8-B store (c0 is a multiple of 8)
      unsigned long long pk = 0;
#pragma unroll
      for (int j = 0; j < 8; ++j) pk |= (unsigned long long)am[j] << (8 * j);
      *reinterpret_cast<unsigned long long*>(amax + op * C + c0) = pk;
    } else {
#pragma unroll
      for (int j = 0; j < CPT; ++j) amax[op * C + c0 + j] = am[j];
    }
  } else {
    VecIO<T, CPT>::load(Y + op * C + c0, o);
#pragma unroll
    for (int j = 0; j < CPT; ++j) o[j] = fmaf(o[j], sc[j], sh[j]);
  }
  float s[CPT];
  VecIO<T, CPT>::load(S + op * C + c0, s);
  if (s2) {
    float a2[CPT], b2[CPT];
    VecIO<float, CPT>::load(s2 + c0, a2);
    VecIO<float, CPT>::load(t2 + c0, b2);
#pragma unroll
    for (int j = 0; j < CPT; ++j) s[j] = fmaf(s[j], a2[j], b2[j]);
  }
#pragma unroll
  for (int j = 0; j < CPT; ++j) o[j] += s[j];
  VecIO<T, CPT>::store(Out + op * C + c0, o);
}

// Pooled block tail per 2 x 2 quad of outputs (2a..2a+1, 2b..2b+1): their four 3 x 3 s2
// windows cover the 5 x 5 input pixels (4a-1..4a+3, 4b-1..4b+3), each loaded once (25
// loads for 4 outputs instead of 36).  Every output visits its window in (ky, kx) order
// with the same first-max rule as tail_fwd_kernel, so out and amax are identical to it.
template <typename T, int CPT>
__global__ __launch_bounds__(256) void tail_pool_quad_kernel(const T* __restrict__ Y, const float* s1, const float* t1,
                                                             const T* __restrict__ S, const float* s2, const float* t2,
                                                             T* __restrict__ Out, unsigned char* __restrict__ amax,
                                                             int N, int H, int W, int C, int OH, int OW) {
  // 32-bit index arithmetic (the launcher checks N * H * W * C < 2^31): row and column offsets formed
  // once each (64-bit products per load were 75 of the thread's quarter-rate multiplies)
  const unsigned CV = (unsigned)C / CPT;
  const unsigned QH = (OH + 1) / 2, QW = (OW + 1) / 2;
  const unsigned g = blockIdx.x * 256u + threadIdx.x;
  if (g >= (unsigned)N * QH * QW * CV) return;
  const unsigned q = g / CV, c0 = (g - q * CV) * CPT;
  const unsigned t = q / QW, qb = q - t * QW;
  const unsigned n = t / QH, qa = t - n * QH;
  float sc[CPT], sh[CPT];
  VecIO<float, CPT>::load(s1 + c0, sc);
  VecIO<float, CPT>::load(t1 + c0, sh);
  // Branch-free loads: out-of-range rows / columns read a clamped (valid) pixel and are masked to
  // -inf, which the strict first-max rule below never selects -- the same result as skipping them,
  // but without a branch per load all 25 loads (and the 4 skip loads) can be in flight at once
  // (with a branch each, every load was its own round trip).
  const int oh0 = 2 * qa, ow0 = 2 * qb;
  unsigned colo[5];
#pragma unroll
  for (int cc = 0; cc < 5; ++cc) colo[cc] = (unsigned)min(max(4 * (int)qb - 1 + cc, 0), W - 1) * C + c0;
  float sv[4][CPT];
#pragma unroll
  for (int o = 0; o < 4; ++o) {
    const int oh = min(oh0 + (o >> 1), OH - 1), ow = min(ow0 + (o & 1), OW - 1);
    VecIO<T, CPT>::load(S + ((n * OH + oh) * OW + ow) * C + c0, sv[o]);
  }
  float m[4][CPT];
  unsigned char am[4][CPT];
#pragma unroll
  for (int o = 0; o < 4; ++o)
#pragma unroll
    for (int j = 0; j < CPT; ++j) {
      m[o][j] = -INFINITY;
      am[o][j] = 0;
    }
#pragma unroll
  for (int r = 0; r < 5; ++r) {
    const int ihr = 4 * (int)qa - 1 + r;
    const bool rok = ihr >= 0 && ihr < H;
    const unsigned rowo = (n * H + (unsigned)min(max(ihr, 0), H - 1)) * W * C;
#pragma unroll
    for (int cc = 0; cc < 5; ++cc) {
      const int iwr = 4 * (int)qb - 1 + cc;
      const bool ok = rok && iwr >= 0 && iwr < W;
      float v[CPT];
      VecIO<T, CPT>::load(Y + rowo + colo[cc], v);
#pragma unroll
      for (int j = 0; j < CPT; ++j) v[j] = ok ? fmaf(v[j], sc[j], sh[j]) : -INFINITY;
#pragma unroll
      for (int oy = 0; oy < 2; ++oy) {
        const int ky = r - 2 * oy;
        if (ky < 0 || ky > 2) continue;
#pragma unroll
        for (int ox = 0; ox < 2; ++ox) {
          const int kx = cc - 2 * ox;
          if (kx < 0 || kx > 2) continue;
          const int o = oy * 2 + ox;
#pragma unroll
          for (int j = 0; j < CPT; ++j)
            if (v[j] > m[o][j] || (v[j] != v[j])) {
              m[o][j] = v[j];
              am[o][j] = (unsigned char)(ky * 3 + kx);
            }
        }
      }
    }
  }
  float a2[CPT], b2[CPT];
  if (s2) {
    VecIO<float, CPT>::load(s2 + c0, a2);
    VecIO<float, CPT>::load(t2 + c0, b2);
  }
#pragma unroll
  for (int o = 0; o < 4; ++o) {
    const int oh = 2 * qa + (o >> 1), ow = 2 * qb + (o & 1);
    if (oh >= OH || ow >= OW) continue;
    const unsigned op = (n * OH + oh) * OW + ow;
    float res[CPT];
#pragma unroll
    for (int j = 0; j < CPT; ++j) res[j] = m[o][j] + (s2 ? fmaf(sv[o][j], a2[j], b2[j]) : sv[o][j]);
    VecIO<T, CPT>::store(Out + op * C + c0, res);
    unsigned long long pk = 0;
#pragma unroll
    for (int j = 0; j < CPT; ++j) pk |= (unsigned long long)am[o][j] << (8 * j);
    *reinterpret_cast<unsigned long long*>(amax + op * C + c0) = pk;
  }
}

// Max-pool backward by gather, per 2 x 2 quad of input pixels (2a..2a+1, 2b..2b+1): the quad
// lies in windows (a..a+1, b..b+1), so each thread loads 4 windows' dOut / argmax once and
// writes 4 pixels (a per-pixel gather loads 2.25 windows per pixel).
// pool_combine: g[py*2+px][j] = the gradient of input pixel (2a+py, 2b+px) from the 4 windows'
// dOut d[k] and argmax bytes am[k] (0xff: window k absent), rounded to T.
template <typename T, int CPT>
XCP_DEV void pool_combine(const float (&d)[4][CPT], const unsigned (&am)[4][2], float (&g)[4][CPT]) {
  auto tap = [&](int k, int j) { return (am[k][j >> 2] >> (8 * (j & 3))) & 0xffu; };
  // pixel (py, px) of the quad: its windows in (oh, ow) order and the tap it has in each
  //   (0,0): w00 t4          (0,1): w00 t5, w01 t3
  //   (1,0): w00 t7, w10 t1  (1,1): w00 t8, w01 t6, w10 t2, w11 t0
#pragma unroll
  for (int py = 0; py < 2; ++py)
#pragma unroll
    for (int px = 0; px < 2; ++px)
#pragma unroll
      for (int j = 0; j < CPT; ++j) {
        float s = 0.f;
        if (tap(0, j) == (unsigned)((1 + py) * 3 + 1 + px)) s += d[0][j];
        if (px && tap(1, j) == (unsigned)((1 + py) * 3)) s += d[1][j];
        if (py && tap(2, j) == (unsigned)(1 + px)) s += d[2][j];
        if (py && px && tap(3, j) == 0u) s += d[3][j];
        g[py * 2 + px][j] = rnd<T>(s);
      }
}

// window k (= dy*2 + dx: (a+dy, b+dx)) of quad (n, a, b): present, and its element offset
// (an absent window maps to window (a, b), so the address is always valid)
XCP_DEV bool pool_win(const PoolSrc& ps, unsigned n, unsigned a, unsigned b, int C, unsigned c0, int k, long& op) {
  const bool ok = (k & 1 ? b + 1 < (unsigned)ps.OW : true) && (k & 2 ? a + 1 < (unsigned)ps.OH : true);
  const unsigned oh = a + (k >> 1), ow = b + (k & 1);
  op = ((long)(n * ps.OH + (ok ? oh : a)) * ps.OW + (ok ? ow : b)) * C + c0;
  return ok;
}

// quad q = (n, a, b): fill g (pool_combine) from dOut / amax (pixels past H / W are left out by
// the callers)
template <typename T, int CPT>
XCP_DEV void pool_quad(const PoolSrc& ps, unsigned n, unsigned a, unsigned b, int C, unsigned c0,
                       float (&g)[4][CPT]) {
  const T* dOut = reinterpret_cast<const T*>(ps.dOut);
  float d[4][CPT];
  unsigned am[4][2];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    long op;
    const bool ok = pool_win(ps, n, a, b, C, c0, k, op);
    VecIO<T, CPT>::load(dOut + op, d[k]);
    const uint2 m = *reinterpret_cast<const uint2*>(ps.amax + op);
    am[k][0] = ok ? m.x : 0xffffffffu;   // 0xff never matches a tap
    am[k][1] = ok ? m.y : 0xffffffffu;
  }
  pool_combine<T, CPT>(d, am, g);
}

// dZ = max-pool backward of dOut (one thread per input quad and 8 channels)
template <typename T, int CPT>
__global__ __launch_bounds__(256) void maxpool_bwd_quad_kernel(PoolSrc ps, T* __restrict__ dZ, int N, int C) {
  const unsigned CV = (unsigned)C / CPT;
  const unsigned gi = blockIdx.x * 256u + threadIdx.x;
  if (gi >= (unsigned)N * ps.OH * ps.OW * CV) return;
  const unsigned q = gi / CV, c0 = (gi - q * CV) * CPT;
  const unsigned t = q / (unsigned)ps.OW, b = q - t * ps.OW;
  const unsigned n = t / (unsigned)ps.OH, a = t - n * ps.OH;
  float g[4][CPT];
  pool_quad<T, CPT>(ps, n, a, b, C, c0, g);
#pragma unroll
  for (int py = 0; py < 2; ++py) {
    if (2 * a + py >= (unsigned)ps.H) break;
#pragma unroll
    for (int px = 0; px < 2; ++px) {
      if (2 * b + px >= (unsigned)ps.W) break;
      VecIO<T, CPT>::store(dZ + ((long)(n * ps.H + 2 * a + py) * ps.W + 2 * b + px) * C + c0, g[py * 2 + px]);
    }
  }
}

// The same, fused with the BatchNorm-backward reduce of the BN that precedes the pool:
// part[P][2][C] = per-chunk (sum dz, sum dz*(y-mean)*invstd) over the stored dz (chanred
// layout, ChanRed over quads).  Software-pipelined: the next quad's raw Y / dOut / argmax words
// (clamped to the chunk, so unconditional) are loaded before the current quad is combined, so a
// slot's quads are not one dependent round trip each.
template <typename T, int CPT>
struct QuadRaw {
  static constexpr int NQ = CPT * (int)sizeof(T) / 16;   // 16-B words per CPT channels
  uint4 y[4][NQ], d[4][NQ];
  uint2 am[4];
};

template <typename T, int CPT>
__global__ __launch_bounds__(256) void maxpool_bwd_red_kernel(ChanRed r, PoolSrc ps, T* __restrict__ dZ,
                                                              const T* __restrict__ Y, const float* mean,
                                                              const float* invstd, float* part) {
  using Q = QuadRaw<T, CPT>;
  const int cchunk = blockIdx.x % r.nch, pchunk = blockIdx.x / r.nch;
  const int lcv = threadIdx.x % r.CVB, slot = threadIdx.x / r.CVB;
  const int cv = cchunk * r.CVB + lcv;
  const int c0 = cv * CPT;
  float acc[2][CPT];
#pragma unroll
  for (int j = 0; j < CPT; ++j) acc[0][j] = acc[1][j] = 0.f;
  if (slot < r.SPB && cv < r.CV) {
    float mu[CPT], is[CPT];
    VecIO<float, CPT>::load(mean + c0, mu);
    VecIO<float, CPT>::load(invstd + c0, is);
    const T* dOut = reinterpret_cast<const T*>(ps.dOut);
    const long rb = (long)pchunk * r.rows_per_chunk, re = min(r.rows, rb + r.rows_per_chunk);
    // Quad coordinates (n, a, b) advance incrementally by SPB quads (one division at the start, not two per
    // quad), and every offset is a 32-bit element offset formed once per quad: the four input pixels
    // and the four pooled positions are the quad's base plus uniform strides (the launcher checks that
    // both tensors have fewer than 2^31 elements).
    const unsigned OH = ps.OH, OW = ps.OW, H = ps.H, W = ps.W, C = r.C;
    auto coords = [&](unsigned q, unsigned& n, unsigned& a, unsigned& b) {
      const unsigned t = q / OW;
      b = q - t * OW;
      n = t / OH;
      a = t - n * OH;
    };
    const unsigned db = (unsigned)r.SPB % OW, da = (unsigned)r.SPB / OW;
    auto advance = [&](unsigned& n, unsigned& a, unsigned& b) {
      b += db;
      a += da;
      if (b >= OW) {
        b -= OW;
        ++a;
      }
      while (a >= OH) {
        a -= OH;
        ++n;
      }
    };
    // input pixel (2a + dy, 2b + dx) of the quad, clamped into the image as the forward's window reads
    auto ybase = [&](unsigned n, unsigned a, unsigned b) { return ((n * H + 2 * a) * W + 2 * b) * C + (unsigned)c0; };
    auto fetch = [&](unsigned q, unsigned n, unsigned a, unsigned b, Q& in) {
      const unsigned y0 = ybase(n, a, b);
      const unsigned sy = 2 * a + 1 < H ? W * C : 0u, sx = 2 * b + 1 < W ? C : 0u;
      const unsigned d0 = q * C + (unsigned)c0;
      const bool okx = b + 1 < OW, oky = a + 1 < OH;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const uint4* src = reinterpret_cast<const uint4*>(Y + y0 + (k & 2 ? sy : 0u) + (k & 1 ? sx : 0u));
#pragma unroll
        for (int i = 0; i < Q::NQ; ++i) in.y[k][i] = src[i];
        const bool ok = (k & 1 ? okx : true) && (k & 2 ? oky : true);   // as pool_win
        const unsigned op = d0 + (ok ? (k & 1 ? C : 0u) + (k & 2 ? OW * C : 0u) : 0u);
        const uint4* dsrc = reinterpret_cast<const uint4*>(dOut + op);
#pragma unroll
        for (int i = 0; i < Q::NQ; ++i) in.d[k][i] = dsrc[i];
        in.am[k] = *reinterpret_cast<const uint2*>(ps.amax + op);
      }
    };
    Q cur;
    long p = rb + slot;
    unsigned n = 0, a = 0, b = 0, nl, al, bl;
    coords((unsigned)(re - 1), nl, al, bl);   // the clamped look-ahead past the chunk
    if (p < re) {
      coords((unsigned)p, n, a, b);
      fetch((unsigned)p, n, a, b, cur);
    }
    for (; p < re; p += r.SPB) {
      unsigned n2 = n, a2 = a, b2 = b;
      advance(n2, a2, b2);
      Q nxt;
      if (p + r.SPB < re) fetch((unsigned)(p + r.SPB), n2, a2, b2, nxt);
      else fetch((unsigned)(re - 1), nl, al, bl, nxt);
      float d[4][CPT], y[4][CPT];
      unsigned am[4][2];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const bool ok = (k & 1 ? b + 1 < OW : true) && (k & 2 ? a + 1 < OH : true);
        VecIO<T, CPT>::load(reinterpret_cast<const T*>(cur.d[k]), d[k]);
        VecIO<T, CPT>::load(reinterpret_cast<const T*>(cur.y[k]), y[k]);
        am[k][0] = ok ? cur.am[k].x : 0xffffffffu;   // 0xff never matches a tap
        am[k][1] = ok ? cur.am[k].y : 0xffffffffu;
      }
      float g[4][CPT];
      pool_combine<T, CPT>(d, am, g);
      const unsigned y0 = ybase(n, a, b);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const unsigned h = 2 * a + (k >> 1), w = 2 * b + (k & 1);
        if (h >= H || w >= W) continue;
        VecIO<T, CPT>::store(dZ + y0 + (k & 2 ? W * C : 0u) + (k & 1 ? C : 0u), g[k]);
#pragma unroll
        for (int j = 0; j < CPT; ++j) {
          acc[0][j] += g[k][j];
          acc[1][j] = fmaf(g[k][j], (y[k][j] - mu[j]) * is[j], acc[1][j]);
        }
      }
      cur = nxt;
      n = n2;
      a = a2;
      b = b2;
    }
  }
  chanred_finish<CPT>(r, acc, part, cchunk, pchunk, lcv, slot);
}

// final: feats[n][c] = mean_{hw} relu(y*s+t)   (fp32 out)
template <typename T>
__global__ __launch_bounds__(256) void avgpool_fwd_kernel(const T* __restrict__ Y, const float* s, const float* t,
                                                          float* __restrict__ F, int N, int HW, int C) {
  const long g = (long)blockIdx.x * 256 + threadIdx.x;
  if (g >= (long)N * C) return;
  const int c = (int)(g % C);
  const int n = (int)(g / C);
  const float sc = s[c], sh = t[c];
  float acc = 0.f;
  for (int p = 0; p < HW; ++p) acc += fmaxf(fmaf(to_f(Y[((long)n * HW + p) * C + c]), sc, sh), 0.f);
  F[g] = acc / (float)HW;
}

// dz[n,p,c] = (y*s+t > 0) ? dF[n][c] / HW : 0
template <typename T, int CPT>
__global__ __launch_bounds__(256) void avgpool_bwd_kernel(const float* __restrict__ dF, const T* __restrict__ Y,
                                                          const float* s, const float* t, T* __restrict__ dZ, int N, int HW,
                                                          int C) {
  const int CV = C / CPT;
  const long g = (long)blockIdx.x * 256 + threadIdx.x;
  if (g >= (long)N * HW * CV) return;
  const int c0 = (int)(g % CV) * CPT;
  const long p = g / CV;
  const int n = (int)(p / HW);
  float y[CPT], sc[CPT], sh[CPT], d[CPT];
  VecIO<T, CPT>::load(Y + p * C + c0, y);
  VecIO<float, CPT>::load(s + c0, sc);
  VecIO<float, CPT>::load(t + c0, sh);
  VecIO<float, CPT>::load(dF + (long)n * C + c0, d);
  const float inv = 1.f / (float)HW;
#pragma unroll
  for (int j = 0; j < CPT; ++j) y[j] = fmaf(y[j], sc[j], sh[j]) > 0.f ? d[j] * inv : 0.f;
  VecIO<T, CPT>::store(dZ + p * C + c0, y);
}

inline unsigned nblk(long n) { return (unsigned)((n + 255) / 256); }

template <typename T, int MODE>
int chanred_launch(long rows, int C, const void* A, const void* B, const float* mean, const float* invstd, float* part,
                   hipStream_t st, const float* ms = nullptr, const float* mt = nullptr) {
  constexpr int CPT = 8;
  if (rows * C >= 0x7fffffffL) return XCP_EUNSUPPORTED;   // 32-bit element offsets in the kernel
  ChanRed r = make_chanred(rows, C, CPT, 1024);
  const long P = chanred_P(r);
  const size_t smem = (size_t)r.SPB * 2 * r.CVB * CPT * sizeof(float);
  hipLaunchKernelGGL((chanred_kernel<T, MODE, CPT>), dim3((unsigned)(P * r.nch)), dim3(256), smem, st, r, A, B, mean,
                     invstd, ms, mt, part);
  return (int)hipGetLastError();
}

inline PoolSrc pool_src(const void* dOut, const unsigned char* amax, int H, int W) {
  return PoolSrc{dOut, amax, H, W, (H - 1) / 2 + 1, (W - 1) / 2 + 1};
}

}  // namespace

extern "C" {

int xcp_colreduce_f32(const float* in, int S, long L, long ld, float* out, int G, int accumulate, hipStream_t st) {
  if (L <= 0) return XCP_OK;
  if (ld < L) return XCP_EINVAL;
  if (G > S) G = S;
  if (G < 1) G = 1;
  if (accumulate && G != 1) return XCP_EINVAL;
  const bool v4 = L % 4 == 0 && ld % 4 == 0 && ((uintptr_t)in % 16) == 0 && ((uintptr_t)out % 16) == 0;
  const long cols_per_block = v4 ? 256 : 64;
  const dim3 grid((unsigned)((L + cols_per_block - 1) / cols_per_block), G);
  if (v4) {
    if (accumulate) hipLaunchKernelGGL((colreduce_kernel<true, 4>), grid, dim3(256), 0, st, in, S, L, ld, out, G);
    else hipLaunchKernelGGL((colreduce_kernel<false, 4>), grid, dim3(256), 0, st, in, S, L, ld, out, G);
  } else {
    if (accumulate) hipLaunchKernelGGL((colreduce_kernel<true, 1>), grid, dim3(256), 0, st, in, S, L, ld, out, G);
    else hipLaunchKernelGGL((colreduce_kernel<false, 1>), grid, dim3(256), 0, st, in, S, L, ld, out, G);
  }
  return (int)hipGetLastError();
}

// jobs: HOST int64 [njobs][7] = (in, out, S, L, ld, G, accumulate) -- njobs <= 16 column
// reductions (each as xcp_colreduce_f32) in one launch; every job needs L % 4 == 0, ld % 4 == 0
// and 16-B aligned in / out
int xcp_colreduce_multi(const long long* jobs, int njobs, hipStream_t st) {
  if (njobs <= 0) return XCP_OK;
  if (njobs > CR_MAXJ) return XCP_EINVAL;
  CRMulti m{};
  int blk = 0, n = 0;
  for (int i = 0; i < njobs; ++i) {
    const long long* r = jobs + 7L * i;
    CRJob j{reinterpret_cast<const float*>(r[0]), reinterpret_cast<float*>(r[1]), (long)r[3], (long)r[4], (int)r[2],
            (int)r[5], (int)r[6], 0, 0};
    if (j.L <= 0) continue;
    if (j.ld < j.L || j.L % 4 || j.ld % 4 || ((uintptr_t)j.in % 16) || ((uintptr_t)j.out % 16)) return XCP_EINVAL;
    if (j.G > j.S) j.G = j.S;
    if (j.G < 1) j.G = 1;
    if (j.acc && j.G != 1) return XCP_EINVAL;
    j.nbx = (int)((j.L + 255) / 256);
    j.blk0 = blk;
    blk += j.nbx * j.G;
    m.j[n++] = j;
  }
  m.njobs = n;
  if (n == 0) return XCP_OK;
  hipLaunchKernelGGL(colreduce_multi_kernel, dim3(blk), dim3(256), 0, st, m);
  return (int)hipGetLastError();
}

// slab groups for the first level of a two-level reduction of S slabs of L floats
// (0 = reduce in one pass): about 1024 workgroups, >= 8 slabs per group, <= 64 groups
int xcp_colreduce_groups(int S, long L) {
  const long blocks = (L + 255) / 256;
  if (S <= 16 || blocks >= 512) return 0;
  long G = 1024 / blocks;
  const long gs = (S + 7) / 8;
  if (G > gs) G = gs;
  if (G > 64) G = 64;
  return G <= 1 ? 0 : (int)G;
}

// number of partial rows the channel reductions below produce
int xcp_chanred_parts(long rows, int C) {
  ChanRed r = make_chanred(rows, C, 8, 1024);
  return (int)chanred_P(r);
}

// part[P][2][C] = per-chunk (sum x, sum x^2) over rows of X[rows][C]
int xcp_row_stats(int dtype, const void* X, long rows, int C, float* part, hipStream_t st) {
  if (C % 8) return XCP_EINVAL;
  if (dtype == XCP_BF16) return chanred_launch<bf16, 0>(rows, C, X, nullptr, nullptr, nullptr, part, st);
  if (dtype == XCP_F32) return chanred_launch<float, 0>(rows, C, X, nullptr, nullptr, nullptr, part, st);
  return XCP_EUNSUPPORTED;
}

// part[P][2][C] = per-chunk (sum dz, sum dz*(y-mean)*invstd)
// ms / mt (may be null): affine of the BN whose ReLU'd output dZ is the gradient of
int xcp_bn_bwd_reduce(int dtype, const void* dZ, const void* Y, const float* mean, const float* invstd, const float* ms,
                      const float* mt, long rows, int C, float* part, hipStream_t st) {
  if (C % 8) return XCP_EINVAL;
  if ((ms == nullptr) != (mt == nullptr)) return XCP_EINVAL;
  if (ms) {
    if (dtype == XCP_BF16) return chanred_launch<bf16, 2>(rows, C, dZ, Y, mean, invstd, part, st, ms, mt);
    if (dtype == XCP_F32) return chanred_launch<float, 2>(rows, C, dZ, Y, mean, invstd, part, st, ms, mt);
    return XCP_EUNSUPPORTED;
  }
  if (dtype == XCP_BF16) return chanred_launch<bf16, 1>(rows, C, dZ, Y, mean, invstd, part, st);
  if (dtype == XCP_F32) return chanred_launch<float, 1>(rows, C, dZ, Y, mean, invstd, part, st);
  return XCP_EUNSUPPORTED;
}

// BatchNorm finalize straight from fp32 partial rows part[R][2][C] (train mode)
int xcp_bn_finalize_part(const float* part, int R, int C, int CP, double count, const float* gamma, const float* beta,
                         float* rmean, float* rvar, float momentum, float eps, float* mean_o, float* invstd_o,
                         float* scale_o, float* shift_o, hipStream_t st) {
  if (C <= 0) return XCP_OK;
  if (R <= 0 || CP < C) return XCP_EINVAL;
  hipLaunchKernelGGL(bn_finalize_part_kernel, dim3((CP + FIN_CH - 1) / FIN_CH), dim3(64 * FIN_WAVES), 0, st, part, R,
                     C, CP, count, gamma, beta, rmean, rvar, momentum, eps, mean_o, invstd_o, scale_o, shift_o);
  return (int)hipGetLastError();
}

int xcp_bn_bwd_finalize_part(const float* part, int R, int C, int CP, double count, const float* gamma,
                             const float* mean, const float* invstd, float* alpha, float* bcoef, float* delta,
                             float* dgamma, float* dbeta, int flags, hipStream_t st) {
  if (C <= 0) return XCP_OK;
  if (R <= 0 || CP < C) return XCP_EINVAL;
  const int acc = flags & XCP_FIN_ACCUMULATE;
  if (flags & XCP_FIN_NARROW)
    hipLaunchKernelGGL(bn_bwd_finalize_part_kernel<FIN_WAVES_NARROW>, dim3((CP + FIN_CH - 1) / FIN_CH),
                       dim3(64 * FIN_WAVES_NARROW), 0, st, part, R, C, CP, count, gamma, mean, invstd, alpha, bcoef,
                       delta, dgamma, dbeta, acc);
  else
    hipLaunchKernelGGL(bn_bwd_finalize_part_kernel<FIN_WAVES>, dim3((CP + FIN_CH - 1) / FIN_CH), dim3(64 * FIN_WAVES),
                       0, st, part, R, C, CP, count, gamma, mean, invstd, alpha, bcoef, delta, dgamma, dbeta, acc);
  return (int)hipGetLastError();
}

int xcp_bn_finalize(const double* part2, int G, int C, int CP, double count, const float* gamma, const float* beta,
                    float* rmean, float* rvar, float momentum, float eps, int train, float* mean, float* invstd,
                    float* scale, float* shift, hipStream_t st) {
  if (C <= 0) return XCP_OK;
  if (CP < C) return XCP_EINVAL;
  hipLaunchKernelGGL(bn_finalize_kernel, dim3((CP + 255) / 256), dim3(256), 0, st, part2, G, C, CP, count, gamma, beta,
                     rmean, rvar, momentum, eps, train, mean, invstd, scale, shift);
  return (int)hipGetLastError();
}

int xcp_bn_act(int dtype, const void* X, void* Y, const float* scale, const float* shift, int relu, long rows, int C,
               hipStream_t st) {
  if (C % 8) return XCP_EINVAL;
  const unsigned g = nblk(rows * (C / 8));
  if (dtype == XCP_BF16)
    hipLaunchKernelGGL((bn_act_kernel<bf16, 8>), dim3(g), dim3(256), 0, st, (const bf16*)X, (bf16*)Y, scale, shift, relu,
                       rows, C);
  else if (dtype == XCP_F32)
    hipLaunchKernelGGL((bn_act_kernel<float, 8>), dim3(g), dim3(256), 0, st, (const float*)X, (float*)Y, scale, shift,
                       relu, rows, C);
  else
    return XCP_EUNSUPPORTED;
  return (int)hipGetLastError();
}

int xcp_bn_act_strided(int dtype, const void* X, void* Y, const float* scale, const float* shift, int relu, int N, int H,
                       int W, int OH, int OW, int S, int C, hipStream_t st) {
  if (C % 8 || S < 1 || (OH - 1) * S >= H || (OW - 1) * S >= W) return XCP_EINVAL;
  const long rows = (long)N * OH * OW;
  if (rows <= 0) return XCP_OK;
  const unsigned g = nblk(rows * (C / 8));
  if (dtype == XCP_BF16)
    hipLaunchKernelGGL((bn_act_strided_kernel<bf16, 8>), dim3(g), dim3(256), 0, st, (const bf16*)X, (bf16*)Y, scale,
                       shift, relu, H, W, OH, OW, S, rows, C);
  else if (dtype == XCP_F32)
    hipLaunchKernelGGL((bn_act_strided_kernel<float, 8>), dim3(g), dim3(256), 0, st, (const float*)X, (float*)Y, scale,
                       shift, relu, H, W, OH, OW, S, rows, C);
  else
    return XCP_EUNSUPPORTED;
  return (int)hipGetLastError();
}

int xcp_bn_bwd_apply(int dtype, const void* dZ, const void* Y, void* dY, const float* alpha, const float* bcoef,
                     const float* delta, const float* ms, const float* mt, long rows, int C, hipStream_t st) {
  if (C % 8) return XCP_EINVAL;
  if ((ms == nullptr) != (mt == nullptr)) return XCP_EINVAL;
  if (rows <= 0) return XCP_OK;
  if (rows * C >= 0x7fffffffL) return XCP_EUNSUPPORTED;   // 32-bit element offsets in the kernel
  // rows per thread: 4 with the mask (5 coefficient vectors), 2 without (3); at 92,416 x 736 bf16
  // 91.5 -> 74 us and 71 -> 71 us against one row per thread (profiles/r02_bnapply_ab.txt)
  const long rq4 = (rows + 3) / 4, rq2 = (rows + 1) / 2;
#define XCP_APPLY(TT, MK)                                                                                       \
  hipLaunchKernelGGL((bn_bwd_apply_kernel<TT, 8, MK, MK ? 4 : 2>), dim3(nblk((MK ? rq4 : rq2) * (C / 8))),    \
                     dim3(256), 0, st, (const TT*)dZ, (const TT*)Y, (TT*)dY, alpha, bcoef, delta, ms, mt, rows, C)
  if (dtype == XCP_BF16) {
    if (ms) XCP_APPLY(bf16, true);
    else XCP_APPLY(bf16, false);
  } else if (dtype == XCP_F32) {
    if (ms) XCP_APPLY(float, true);
    else XCP_APPLY(float, false);
  } else
#undef XCP_APPLY
    return XCP_EUNSUPPORTED;
  return (int)hipGetLastError();
}

int xcp_relu_bwd(int dtype, void* dX, const void* X, long rows, int C, hipStream_t st) {
  if (C % 8) return XCP_EINVAL;
  const unsigned g = nblk(rows * (C / 8));
  if (dtype == XCP_BF16)
    hipLaunchKernelGGL((relu_bwd_kernel<bf16, 8>), dim3(g), dim3(256), 0, st, (bf16*)dX, (const bf16*)X, rows, C);
  else if (dtype == XCP_F32)
    hipLaunchKernelGGL((relu_bwd_kernel<float, 8>), dim3(g), dim3(256), 0, st, (float*)dX, (const float*)X, rows, C);
  else
    return XCP_EUNSUPPORTED;
  return (int)hipGetLastError();
}

int xcp_tail_fwd(int dtype, const void* Y, const float* s1, const float* t1, int pool, const void* S, const float* s2,
                 const float* t2, void* Out, unsigned char* amax, int N, int H, int W, int C, hipStream_t st) {
  if (C % 8) return XCP_EINVAL;
  const int OH = pool ? (H - 1) / 2 + 1 : H, OW = pool ? (W - 1) / 2 + 1 : W;
  if (pool) {   // one thread per 2 x 2 output quad x 8 channels
    if ((long)N * H * W * C >= 0x7fffffffL) return XCP_EUNSUPPORTED;   // 32-bit element offsets in the kernel
    const unsigned gq = nblk((long)N * ((OH + 1) / 2) * ((OW + 1) / 2) * (C / 8));
    if (dtype == XCP_BF16)
      hipLaunchKernelGGL((tail_pool_quad_kernel<bf16, 8>), dim3(gq), dim3(256), 0, st, (const bf16*)Y, s1, t1,
                         (const bf16*)S, s2, t2, (bf16*)Out, amax, N, H, W, C, OH, OW);
    else if (dtype == XCP_F32)
      hipLaunchKernelGGL((tail_pool_quad_kernel<float, 8>), dim3(gq), dim3(256), 0, st, (const float*)Y, s1, t1,
                         (const float*)S, s2, t2, (float*)Out, amax, N, H, W, C, OH, OW);
    else
      return XCP_EUNSUPPORTED;
    return (int)hipGetLastError();
  }
  if ((long)N * H * W * C >= 0x7fffffffL) return XCP_EUNSUPPORTED;   // 32-bit element offsets in the kernel
  const unsigned g = nblk((long)N * OH * OW * (C / 8));
  if (dtype == XCP_BF16)
    hipLaunchKernelGGL((tail_fwd_kernel<bf16, 8>), dim3(g), dim3(256), 0, st, (const bf16*)Y, s1, t1, pool,
                       (const bf16*)S, s2, t2, (bf16*)Out, amax, N, H, W, C, OH, OW);
  else if (dtype == XCP_F32)
    hipLaunchKernelGGL((tail_fwd_kernel<float, 8>), dim3(g), dim3(256), 0, st, (const float*)Y, s1, t1, pool,
                       (const float*)S, s2, t2, (float*)Out, amax, N, H, W, C, OH, OW);
  else
    return XCP_EUNSUPPORTED;
  return (int)hipGetLastError();
}

int xcp_maxpool_bwd(int dtype, const void* dOut, const unsigned char* amax, void* dZ, int N, int H, int W, int C,
                    hipStream_t st) {
  if (C % 8) return XCP_EINVAL;
  const PoolSrc ps = pool_src(dOut, amax, H, W);
  const unsigned g = nblk((long)N * ps.OH * ps.OW * (C / 8));
  if (dtype == XCP_BF16)
    hipLaunchKernelGGL((maxpool_bwd_quad_kernel<bf16, 8>), dim3(g), dim3(256), 0, st, ps, (bf16*)dZ, N, C);
  else if (dtype == XCP_F32)
    hipLaunchKernelGGL((maxpool_bwd_quad_kernel<float, 8>), dim3(g), dim3(256), 0, st, ps, (float*)dZ, N, C);
  else
    return XCP_EUNSUPPORTED;
  return (int)hipGetLastError();
}

// partial rows (P) of xcp_maxpool_bwd_bnred
int xcp_maxpool_bwd_bnred_parts(int N, int H, int W, int C) {
  const long quads = (long)N * ((H - 1) / 2 + 1) * ((W - 1) / 2 + 1);
  return (int)chanred_P(make_chanred(quads, C, 8, 1024));
}

// xcp_maxpool_bwd + the BN-backward reduce of its output against Y [N][H][W][C] in one pass:
// part[P][2][C] = (sum dz, sum dz*(y-mean)*invstd) partials, as xcp_bn_bwd_reduce
int xcp_maxpool_bwd_bnred(int dtype, const void* dOut, const unsigned char* amax, void* dZ, const void* Y,
                          const float* mean, const float* invstd, int N, int H, int W, int C, float* part,
                          hipStream_t st) {
  if (C % 8) return XCP_EINVAL;
  if ((long)N * H * W * C >= 0x7fffffffL) return XCP_EUNSUPPORTED;   // 32-bit element offsets in the kernel
  const PoolSrc ps = pool_src(dOut, amax, H, W);
  const ChanRed r = make_chanred((long)N * ps.OH * ps.OW, C, 8, 1024);
  const long P = chanred_P(r);
  const size_t smem = (size_t)r.SPB * 2 * r.CVB * 8 * sizeof(float);
  if (dtype == XCP_BF16)
    hipLaunchKernelGGL((maxpool_bwd_red_kernel<bf16, 8>), dim3((unsigned)(P * r.nch)), dim3(256), smem, st, r, ps,
                       (bf16*)dZ, (const bf16*)Y, mean, invstd, part);
  else if (dtype == XCP_F32)
    hipLaunchKernelGGL((maxpool_bwd_red_kernel<float, 8>), dim3((unsigned)(P * r.nch)), dim3(256), smem, st, r, ps,
                       (float*)dZ, (const float*)Y, mean, invstd, part);
  else
    return XCP_EUNSUPPORTED;
  return (int)hipGetLastError();
}

int xcp_avgpool_fwd(int dtype, const void* Y, const float* s, const float* t, float* F, int N, int HW, int C,
                    hipStream_t st) {
  const unsigned g = nblk((long)N * C);
  if (dtype == XCP_BF16)
    hipLaunchKernelGGL(avgpool_fwd_kernel<bf16>, dim3(g), dim3(256), 0, st, (const bf16*)Y, s, t, F, N, HW, C);
  else if (dtype == XCP_F32)
    hipLaunchKernelGGL(avgpool_fwd_kernel<float>, dim3(g), dim3(256), 0, st, (const float*)Y, s, t, F, N, HW, C);
  else
    return XCP_EUNSUPPORTED;
  return (int)hipGetLastError();
}

int xcp_avgpool_bwd(int dtype, const float* dF, const void* Y, const float* s, const float* t, void* dZ, int N, int HW,
                    int C, hipStream_t st) {
  if (C % 8) return XCP_EINVAL;
  const unsigned g = nblk((long)N * HW * (C / 8));
  if (dtype == XCP_BF16)
    hipLaunchKernelGGL((avgpool_bwd_kernel<bf16, 8>), dim3(g), dim3(256), 0, st, dF, (const bf16*)Y, s, t, (bf16*)dZ, N,
                       HW, C);
  else if (dtype == XCP_F32)
    hipLaunchKernelGGL((avgpool_bwd_kernel<float, 8>), dim3(g), dim3(256), 0, st, dF, (const float*)Y, s, t, (float*)dZ,
                       N, HW, C);
  else
    return XCP_EUNSUPPORTED;
  return (int)hipGetLastError();
}

}  // extern "C"
