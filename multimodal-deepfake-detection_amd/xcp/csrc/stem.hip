// Entry-flow stem conv1 (3->32, 3x3, stride 2, pad 0, no bias) forward and
// weight gradient, plus the small permute/cast kernels used to pack fp32
// master weights into kernel layouts every step.
//
// Reference ops: Xception.conv1 = nn.Conv2d(3, 32, 3, 2, 0, bias=False)
// (Xception.py:118, called at :168); the input is the NCHW fp32 frame batch
// produced by XceptionLSTMV.extract_features (XceptionLSTMV.py:55).  The second
// stem conv (32->64, Xception.py:122) runs on the MFMA GEMM with an im2col row
// gather (gemm.hip, gather modes 2/3).
#include "common.h"

namespace {

constexpr int C1 = 32, K1 = 27;   // conv1 output channels, 3*3*3 taps

// Y[n,oh,ow,co] = sum_{ci,ky,kx} X[n,ci,2oh+ky,2ow+kx] * W[co,ci,ky,kx]
// thread = (output pixel, 8 output channels); W is read through the scalar cache.
template <typename T>
__global__ __launch_bounds__(256) void conv1_fwd_kernel(const float* __restrict__ X, const float* __restrict__ Wt,
                                                        T* __restrict__ Y, int N, int IH, int IW, int OH, int OW) {
  const long g = (long)blockIdx.x * 256 + threadIdx.x;
  const long total = (long)N * OH * OW * (C1 / 8);
  if (g >= total) return;
  const int cg = (int)(g % (C1 / 8));
  const long p = g / (C1 / 8);
  const int ow = (int)(p % OW);
  const long t = p / OW;
  const int oh = (int)(t % OH);
  const int n = (int)(t / OH);
  float xin[K1];
#pragma unroll
  for (int ci = 0; ci < 3; ++ci)
#pragma unroll
    for (int ky = 0; ky < 3; ++ky)
#pragma unroll
      for (int kx = 0; kx < 3; ++kx)
        xin[ci * 9 + ky * 3 + kx] = X[(((long)n * 3 + ci) * IH + (oh * 2 + ky)) * IW + (ow * 2 + kx)];
  float o[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float* w = Wt + (cg * 8 + j) * K1;
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < K1; ++k) s = fmaf(xin[k], w[k], s);
    o[j] = s;
  }
  VecIO<T, 8>::store(Y + p * C1 + cg * 8, o);
}

// dW partial: part[blk][co*27+k] = sum over the block's pixels dY[p][co] * patch[p][k]
template <typename T>
__global__ __launch_bounds__(256) void conv1_wgrad_kernel(const float* __restrict__ X, const T* __restrict__ dY,
                                                          float* __restrict__ part, int N, int IH, int IW, int OH, int OW,
                                                          long pix_per_block) {
  __shared__ float sdy[64][C1 + 1];
  __shared__ float sx[64][K1 + 1];
  const int tid = threadIdx.x;
  const int co = tid & 31, kg = tid >> 5;   // outputs (co, k) for k = kg + 8*i
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
  const long P = (long)N * OH * OW;
  const long pb = (long)blockIdx.x * pix_per_block, pe = min(P, pb + pix_per_block);
  for (long p0 = pb; p0 < pe; p0 += 64) {
    // stage 64 pixels of dY (64x32) and their input patches (64x27)
    for (int i = tid; i < 64 * C1; i += 256) {
      const int pp = i / C1, c = i % C1;
      const long p = p0 + pp;
      sdy[pp][c] = p < pe ? to_f(dY[p * C1 + c]) : 0.f;
    }
    for (int i = tid; i < 64 * K1; i += 256) {
      const int pp = i / K1, k = i % K1;
      const long p = p0 + pp;
      float v = 0.f;
      if (p < pe) {
        const int ow = (int)(p % OW);
        const long t = p / OW;
        const int oh = (int)(t % OH);
        const int n = (int)(t / OH);
        const int ci = k / 9, ky = (k % 9) / 3, kx = k % 3;
        v = X[(((long)n * 3 + ci) * IH + (oh * 2 + ky)) * IW + (ow * 2 + kx)];
      }
      sx[pp][k] = v;
    }
    __syncthreads();
#pragma unroll 4
    for (int pp = 0; pp < 64; ++pp) {
      const float d = sdy[pp][co];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int k = kg + 8 * i;
        if (k < K1) acc[i] = fmaf(d, sx[pp][k], acc[i]);
      }
    }
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int k = kg + 8 * i;
    if (k < K1) part[(long)blockIdx.x * (C1 * K1) + co * K1 + k] = acc[i];
  }
}

// out[perm(i0,i1,i2)] = cast(in[i0][i1][i2]); perm gives, for each output axis, the
// input axis it comes from.
template <typename TO>
__global__ __launch_bounds__(256) void permute3_kernel(const float* __restrict__ in, TO* __restrict__ out, int d0, int d1,
                                                       int d2, int p0, int p1, int p2) {
  const long total = (long)d0 * d1 * d2;
  const long g = (long)blockIdx.x * 256 + threadIdx.x;
  if (g >= total) return;
  const int dims[3] = {d0, d1, d2};
  const int od1 = dims[p1], od2 = dims[p2];
  const int o2 = (int)(g % od2);
  const long t = g / od2;
  const int o1 = (int)(t % od1);
  const int o0 = (int)(t / od1);
  int idx[3];
  idx[p0] = o0;
  idx[p1] = o1;
  idx[p2] = o2;
  out[g] = from_f<TO>(in[((long)idx[0] * d1 + idx[1]) * d2 + idx[2]]);
}

// Many permute3 jobs in one launch (the per-step weight packing of every layer).  jobs is a
// device array of [njobs][12] int64: in, out, d0, d1, d2, p0, p1, p2, out dtype, first block,
// s0, s1 (output strides of the first two output axes: padded layouts).  Workgroup b finds its
// job by binary search over the first-block column (uniform per block).
//
// Every permutation the packs use is a copy or a (batched) 2-D transpose of rows of a
// contiguous fp32 array: those run as 32 x 32 tiles (coalesced reads and writes, the transpose
// through LDS), with the index arithmetic once per workgroup; anything else falls back to one
// element per thread.  A per-element form with 64-bit division for every element took 114 us
// per pack of the 21 M parameters (two per step).
constexpr int PJ = 12;

struct PermPlan {
  int mode;                  // 0 copy, 1 transpose, 2 per element
  int B, R, Cc;              // batch of [R][Cc] fp32 input rows
  long ib, ob, ors;          // input batch stride, output batch stride, output row stride
  int tiles() const { return B * ((R + 31) / 32) * ((Cc + 31) / 32); }
};

__host__ __device__ inline PermPlan perm_plan(int d0, int d1, int d2, int p0, int p1, int p2, long s0, long s1) {
  PermPlan q{2, 1, 0, 0, 0, 0, 0};
  const int od1 = p1 == 0 ? d0 : p1 == 1 ? d1 : d2, od2 = p2 == 0 ? d0 : p2 == 1 ? d1 : d2;
  if (s1 != od2) return q;
  if (p0 == 0 && p1 == 1 && p2 == 2) {   // out[i0][i1 i2] (row pitch s0)
    q = PermPlan{0, 1, d0, d1 * d2, 0, 0, s0};
  } else if (p0 == 1 && p1 == 0 && p2 == 2 && d2 == 1) {   // out[i1][i0]
    q = PermPlan{1, 1, d0, d1, 0, 0, s0};
  } else if (p0 == 0 && p1 == 2 && p2 == 1) {   // out[i0][i2][i1]: d0 transposes of [d1][d2]
    q = PermPlan{1, d0, d1, d2, (long)d1 * d2, s0, s1};
  } else if (p0 == 1 && p1 == 2 && p2 == 0 && s0 == (long)od1 * od2) {   // out[i1 i2][i0]
    q = PermPlan{1, 1, d0, d1 * d2, 0, 0, d0};
  }
  (void)od1;
  return q;
}

XCP_DEV inline void store_as(int dtype, void* out, long o, float v) {
  if (dtype == XCP_BF16) reinterpret_cast<bf16*>(out)[o] = (bf16)v;
  else reinterpret_cast<float*>(out)[o] = v;
}

// four consecutive elements (o a multiple of 4): one 8-B (bf16) or 16-B (fp32) store, the same
// per-element conversion as store_as
XCP_DEV inline void store4_as(int dtype, void* out, long o, float4 v) {
  if (dtype == XCP_BF16) {
    *reinterpret_cast<uint2*>(reinterpret_cast<bf16*>(out) + o) = make_uint2(pk_bf16(v.x, v.y), pk_bf16(v.z, v.w));
  } else {
    *reinterpret_cast<float4*>(reinterpret_cast<float*>(out) + o) = v;
  }
}

__global__ __launch_bounds__(256) void permute3_batch_kernel(const long long* __restrict__ jobs, int njobs) {
  __shared__ float tile[32][33];
  const int b = blockIdx.x;
  int lo = 0, hi = njobs - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (jobs[(long)mid * PJ + 9] <= b) lo = mid;
    else hi = mid - 1;
  }
  const long long* j = jobs + (long)lo * PJ;
  const float* in = reinterpret_cast<const float*>(j[0]);
  void* out = reinterpret_cast<void*>(j[1]);
  const int d0 = (int)j[2], d1 = (int)j[3], d2 = (int)j[4], p0 = (int)j[5], p1 = (int)j[6], p2 = (int)j[7];
  const int dtype = (int)j[8];
  const PermPlan q = perm_plan(d0, d1, d2, p0, p1, p2, j[10], j[11]);
  const int lb = b - (int)j[9];
  if (q.mode == 2) {   // per element
    const long total = (long)d0 * d1 * d2;
    const long g = (long)lb * 256 + threadIdx.x;
    if (g >= total) return;
    const int dims[3] = {d0, d1, d2};
    const int od1 = dims[p1], od2 = dims[p2];
    const int o2 = (int)(g % od2);
    const long t = g / od2;
    const int o1 = (int)(t % od1);
    const int o0 = (int)(t / od1);
    int idx[3];
    idx[p0] = o0;
    idx[p1] = o1;
    idx[p2] = o2;
    store_as(dtype, out, (long)o0 * j[10] + (long)o1 * j[11] + o2, in[((long)idx[0] * d1 + idx[1]) * d2 + idx[2]]);
    return;
  }
  const int ntr = (q.R + 31) / 32, ntc = (q.Cc + 31) / 32;
  const int bb = lb / (ntr * ntc), rem = lb - bb * (ntr * ntc), tr = rem / ntc, tc = rem - tr * ntc;
  const float* src = in + bb * q.ib;
  const long obase = bb * q.ob;
  // rows of 4-element groups (16-B loads, 8-B bf16 / 16-B fp32 stores) whenever the input row length,
  // the output pitch, the per-batch strides, the tile's edge and both base addresses keep every
  // group aligned; per element otherwise (offset views, odd pitches)
  const unsigned long oal = dtype == XCP_BF16 ? 7ul : 15ul;
  const bool vec = (q.Cc & 3) == 0 && (q.ors & 3) == 0 && (q.R & 3) == 0 && (q.ib & 3) == 0 && (q.ob & 3) == 0 &&
                   (reinterpret_cast<unsigned long>(in) & 15ul) == 0 && (reinterpret_cast<unsigned long>(out) & oal) == 0;
  if (vec) {
    const int t8 = threadIdx.x & 7, tr32 = threadIdx.x >> 3;   // 32 rows x 8 four-element groups
    const int r = tr * 32 + tr32, c4 = tc * 32 + t8 * 4;
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (r < q.R && c4 < q.Cc) v = *reinterpret_cast<const float4*>(src + (long)r * q.Cc + c4);
    if (q.mode == 0) {
      if (r < q.R && c4 < q.Cc) store4_as(dtype, out, obase + r * q.ors + c4, v);
      return;
    }
    tile[tr32][t8 * 4] = v.x;
    tile[tr32][t8 * 4 + 1] = v.y;
    tile[tr32][t8 * 4 + 2] = v.z;
    tile[tr32][t8 * 4 + 3] = v.w;
    __syncthreads();
    const int oc = tc * 32 + tr32, orow4 = tr * 32 + t8 * 4;   // output row = input column
    if (oc < q.Cc && orow4 < q.R)
      store4_as(dtype, out, obase + oc * q.ors + orow4,
                make_float4(tile[t8 * 4][tr32], tile[t8 * 4 + 1][tr32], tile[t8 * 4 + 2][tr32], tile[t8 * 4 + 3][tr32]));
    return;
  }
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  const int c = tc * 32 + tx;
  if (q.mode == 0) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int r = tr * 32 + ty + 8 * k;
      if (r < q.R && c < q.Cc) store_as(dtype, out, obase + r * q.ors + c, src[(long)r * q.Cc + c]);
    }
    return;
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int r = tr * 32 + ty + 8 * k;
    tile[ty + 8 * k][tx] = (r < q.R && c < q.Cc) ? src[(long)r * q.Cc + c] : 0.f;
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int oc = tc * 32 + ty + 8 * k, orow = tr * 32 + tx;   // output row = input column
    if (oc < q.Cc && orow < q.R) store_as(dtype, out, obase + oc * q.ors + orow, tile[tx][ty + 8 * k]);
  }
}

// ---------------------------------------------------------------------------------
// Tiled conv1 (default).  The per-pixel kernels above re-read each input value ~9x
// through L1 with scalar stride-2 loads and, in the forward, fetch the 864 weights
// per thread with vector loads; both measured ~0.45 TB/s.  Here a workgroup stages
// the 2*TH+1 input rows (3 channels, fp32) of TH output rows of one frame in LDS with
// coalesced loads.  Forward: a thread computes all 32 channels of one output pixel,
// channel pairs with packed FMAs, weights through the scalar cache (uniform
// addresses).  Weight gradient: a thread owns one output-channel pair x all 27 taps
// (27 packed accumulators) for every 16th pixel of the tile, loops over tiles
// (persistent), and the 16 pixel groups are reduced in LDS at the end.
typedef float f2v __attribute__((ext_vector_type(2)));

// LDS row pitch of the staged input (floats): IW rounded up to 64 (one 4-B LDS-DMA
// instruction fills 64 consecutive floats of a row)
XCP_DEV int pitch1(int IW) { return (IW + 63) & ~63; }
__device__ float g_zero1[64];

// Stage the 3 x (2*TH+1) input rows of output rows [oh0, oh0+TH) with 4-B LDS-DMA
// (wave w fills rows w, w+4, ...; all issued before one wait).  Rows past the frame
// and columns past IW read zeros.
template <int TH>
XCP_DEV void stage_rows(const float* __restrict__ X, float* sx, int n, int oh0, int IH, int IW, int tid) {
  constexpr int R = 2 * TH + 1;
  const int rows = min(R, IH - 2 * oh0), P = pitch1(IW);
  const int lane = tid & 63, w = tid >> 6;
  for (int rr = w; rr < 3 * R; rr += 4) {
    const int ci = rr / R, r = rr - ci * R;
    const float* src = X + (((long)n * 3 + ci) * IH + 2 * oh0 + r) * IW;
    for (int j = 0; j < P; j += 64) {
      const int col = j + lane;
      const float* p = (r < rows && col < IW) ? src + col : g_zero1 + lane;
      __builtin_amdgcn_global_load_lds((const void __attribute__((address_space(1)))*)p,
                                       (void __attribute__((address_space(3)))*)(sx + rr * P + j), 4, 0, 0);
    }
  }
}

template <typename T, int TH>
__global__ __launch_bounds__(256) void conv1_fwd_tile_kernel(const float* __restrict__ X, const float* __restrict__ Wt,
                                                             T* __restrict__ Y, int N, int IH, int IW, int OH, int OW) {
  extern __shared__ __attribute__((aligned(16))) float sx[];   // [3][2*TH+1][pitch] input, then [27][32] weights
  constexpr int R = 2 * TH + 1;
  const int P = pitch1(IW);
  float* sw = sx + 3 * R * P;
  const int ntile = (OH + TH - 1) / TH;
  const int n = blockIdx.x / ntile, oh0 = (blockIdx.x % ntile) * TH;
  const int tid = threadIdx.x;
  stage_rows<TH>(X, sx, n, oh0, IH, IW, tid);
  for (int i = tid; i < C1 * K1; i += 256) sw[(i % K1) * C1 + i / K1] = Wt[i];   // [co][k] -> [k][co]
  __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0): this wave's LDS-DMA landed (then the barrier)
  __syncthreads();
  const int npx = min(TH, OH - oh0) * OW;
  // two pixels per thread and pass; taps outer, the 32 weights of a tap read from LDS
  // (one address for the whole wave: broadcast), channel pairs x pixel pairs packed
  for (int p0 = 2 * tid; p0 < npx; p0 += 512) {
    const int p1 = min(p0 + 1, npx - 1);
    const int r0 = p0 / OW, r1 = p1 / OW;
    const int b0 = 2 * r0 * P + 2 * (p0 - r0 * OW), b1 = 2 * r1 * P + 2 * (p1 - r1 * OW);
    f2v acc[C1];   // acc[co] = (pixel p0, pixel p1)
#pragma unroll
    for (int co = 0; co < C1; ++co) acc[co] = f2v(0.f);
#pragma unroll 3
    for (int k = 0; k < K1; ++k) {
      const int ci = k / 9, ky = (k % 9) / 3, kx = k % 3;
      const int off = (ci * R + ky) * P + kx;
      const f2v x{sx[b0 + off], sx[b1 + off]};
      const float4* wk = reinterpret_cast<const float4*>(sw + k * C1);
#pragma unroll
      for (int q = 0; q < C1 / 4; ++q) {
        const float4 w4 = wk[q];
        acc[4 * q + 0] = __builtin_elementwise_fma(x, f2v(w4.x), acc[4 * q + 0]);
        acc[4 * q + 1] = __builtin_elementwise_fma(x, f2v(w4.y), acc[4 * q + 1]);
        acc[4 * q + 2] = __builtin_elementwise_fma(x, f2v(w4.z), acc[4 * q + 2]);
        acc[4 * q + 3] = __builtin_elementwise_fma(x, f2v(w4.w), acc[4 * q + 3]);
      }
    }
    float o[C1];
#pragma unroll
    for (int co = 0; co < C1; ++co) o[co] = acc[co][0];
    T* yp = Y + ((long)n * OH * OW + (long)oh0 * OW + p0) * C1;
#pragma unroll
    for (int q = 0; q < C1; q += 8) VecIO<T, 8>::store(yp + q, o + q);
    if (p0 + 1 < npx) {
#pragma unroll
      for (int co = 0; co < C1; ++co) o[co] = acc[co][1];
#pragma unroll
      for (int q = 0; q < C1; q += 8) VecIO<T, 8>::store(yp + C1 + q, o + q);
    }
  }
}

constexpr int W1_TH = 2;

template <typename T>
__global__ __launch_bounds__(256) void conv1_wgrad_tile_kernel(const float* __restrict__ X, const T* __restrict__ dY,
                                                               float* __restrict__ part, int N, int IH, int IW, int OH,
                                                               int OW) {
  constexpr int TH = W1_TH, R = 2 * TH + 1;
  extern __shared__ __attribute__((aligned(16))) float sm1[];   // input [3][R][pitch] fp32, then dY [TH*OW][C1] (T)
  const int P = pitch1(IW);
  float* sx = sm1;
  T* sdy = reinterpret_cast<T*>(sm1 + 3 * R * P);   // 3*R*P floats: a multiple of 4 -> 16-B aligned
  const int tid = threadIdx.x, cq = tid & 7, pg = tid >> 3;   // channels 4cq..4cq+3; 32 pixel groups
  const int ntile = (OH + TH - 1) / TH;
  f2v acc[2][K1];   // [channel pair][tap]
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int k = 0; k < K1; ++k) acc[h][k] = f2v(0.f);
  for (int t = blockIdx.x; t < N * ntile; t += gridDim.x) {
    const int n = t / ntile, oh0 = (t % ntile) * TH;
    const int npx = min(TH, OH - oh0) * OW;
    __syncthreads();   // previous tile consumed
    stage_rows<TH>(X, sx, n, oh0, IH, IW, tid);
    {   // dY rows of the tile: contiguous [npx][32] in NHWC, 16-B LDS-DMA
      const T* src = dY + (((long)n * OH + oh0) * OW) * C1;
      constexpr int EPC = 16 / (int)sizeof(T);
      const int chunks = npx * C1 / EPC;
      const int lane = tid & 63;
      for (int i0 = (tid >> 6) * 64; i0 < chunks; i0 += 256) {
        const bool ok = i0 + lane < chunks;
        const void* p = ok ? (const void*)(src + (long)(i0 + lane) * EPC) : (const void*)g_zero1;
        if (ok)
          __builtin_amdgcn_global_load_lds((const void __attribute__((address_space(1)))*)p,
                                           (void __attribute__((address_space(3)))*)(reinterpret_cast<char*>(sdy) +
                                                                                     (long)i0 * 16),
                                           16, 0, 0);
      }
    }
    __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0)
    __syncthreads();
    for (int p = pg; p < npx; p += 32) {
      const int r = p / OW, ow = p - r * OW;
      float d[4];
      VecIO<T, 4>::load(sdy + p * C1 + 4 * cq, d);
      const f2v d0{d[0], d[1]}, d1{d[2], d[3]};
      const float* xb = sx + 2 * r * P + 2 * ow;
#pragma unroll
      for (int ci = 0; ci < 3; ++ci)
#pragma unroll
        for (int ky = 0; ky < 3; ++ky) {
          const float* xr = xb + (ci * R + ky) * P;
          const float2 x01 = *reinterpret_cast<const float2*>(xr);
          const float x2 = xr[2];
          const int k = ci * 9 + ky * 3;
          acc[0][k] = __builtin_elementwise_fma(f2v(x01.x), d0, acc[0][k]);
          acc[1][k] = __builtin_elementwise_fma(f2v(x01.x), d1, acc[1][k]);
          acc[0][k + 1] = __builtin_elementwise_fma(f2v(x01.y), d0, acc[0][k + 1]);
          acc[1][k + 1] = __builtin_elementwise_fma(f2v(x01.y), d1, acc[1][k + 1]);
          acc[0][k + 2] = __builtin_elementwise_fma(f2v(x2), d0, acc[0][k + 2]);
          acc[1][k + 2] = __builtin_elementwise_fma(f2v(x2), d1, acc[1][k + 2]);
        }
    }
  }
  // reduce the 32 pixel groups: lanes xor 8 / 16 / 32 within the wave, then the 4 waves in LDS
  __syncthreads();
  float* red = sm1;   // [4 waves][C1][K1]
  const int w = tid >> 6;
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int k = 0; k < K1; ++k)
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        float v = acc[h][k][e];
        v += __shfl_xor(v, 8, 64);
        v += __shfl_xor(v, 16, 64);
        v += __shfl_xor(v, 32, 64);
        if ((tid & 63) < 8) red[(w * C1 + 4 * cq + 2 * h + e) * K1 + k] = v;
      }
  __syncthreads();
  for (int i = tid; i < C1 * K1; i += 256) {
    float v = 0.f;
#pragma unroll
    for (int q = 0; q < 4; ++q) v += red[q * C1 * K1 + i];
    part[(long)blockIdx.x * (C1 * K1) + i] = v;
  }
}

constexpr int W1R_IW = 320;                          // widest frame: 9 input rows of pitch 320 floats
constexpr int W1R_OW = (W1R_IW - 3) / 2 + 1;         // 159 output pixels -> 636 16-B chunks per row
constexpr int W1R_OWM = W1R_OW;
constexpr int W1R_DL = (W1R_OW * 4 + 255) / 256;     // 16-B output(-gradient) chunks per thread and tile (3)

// The nine stride-2 input rows (3 channels x 3 kernel rows) of one output row, fetched as 16-B
// chunks: chunk e = tid + 256 k (k < 3) of the tile is row e / C4, columns 4 (e % C4) .. +3, the last
// chunk of a row clamped to end at column IW - 1 (it rewrites three columns of its neighbour with the
// same values).  Frame rows are 299 floats (no 16-B alignment): 4-B aligned dwordx4 loads.  One
// 16-B load per lane instead of four 4-B ones (load issue, not bytes, bounds a 4-B-lane stream:
// MI355X_MICROARCH "store tail ... 8x dwordx4 halves it").
typedef float f4a4 __attribute__((ext_vector_type(4), aligned(4)));
struct XRowChunks {
  int off[3];   // element offset inside the frame's [3][IH][IW] block, relative to input row 2 oh
  int lds[3];   // LDS float index (< 0: no chunk)
};
XCP_DEV XRowChunks xrow_chunks(int tid, int IH, int IW, int P) {
  const int C4 = (IW + 3) / 4;
  XRowChunks m;
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const int e = tid + 256 * k, r = e / C4, j = e - r * C4;
    const int col = min(4 * j, IW - 4);
    const bool ok = r < 9;
    m.off[k] = ok ? (r / 3) * IH * IW + (r % 3) * IW + col : 0;
    m.lds[k] = ok ? r * P + col : -1;
  }
  return m;
}
XCP_DEV void xrow_fetch(const float* xb, const XRowChunks& m, f4a4 (&rx)[3]) {
#pragma unroll
  for (int k = 0; k < 3; ++k) rx[k] = *reinterpret_cast<const f4a4*>(xb + m.off[k]);
}
XCP_DEV void xrow_store(float* sx, const XRowChunks& m, const f4a4 (&rx)[3]) {
#pragma unroll
  for (int k = 0; k < 3; ++k)
    if (m.lds[k] >= 0) {
#pragma unroll
      for (int i = 0; i < 4; ++i) sx[m.lds[k] + i] = rx[k][i];   // (clamped chunks: not 16-B aligned)
    }
}

// Forward over one output row per tile (bf16 output, frames up to W1R_IW wide; see the weight-gradient
// row kernel below for the tile and the register prefetch), with BN1's batch statistics (STATS): each
// workgroup sums y and y^2 of the stored (bf16-rounded) outputs of its tiles per channel and writes one
// partial row part[blockIdx][2][32] -- the per-channel reduce pass over the 364 MB output is gone.
// The convolution is an im2col product on the matrix cores: per 16 output pixels and 16 channels,
// v_mfma_f32_16x16x32_bf16 over A = the pixels' 27 inputs (padded to 32, gathered from the staged rows)
// and B = the 32 x 27 kernel (in registers), each split into a bf16 head and a bf16 tail (x = hi + lo,
// |lo| <= 2^-9 |x|): hi.hi + lo.hi + hi.lo in fp32, three MFMAs, products exact to ~2^-17 -- the fp32
// conv's accuracy, not bf16's (a single bf16 x bf16 product moved the 64^2 features' cosine to the
// fp32 reference from 0.9991 to 0.9988).  The fp32 FMA form (27 packed FMAs and 18 LDS reads per pixel
// and channel pair) was bound by LDS issue at ~2.4 TB/s; the matrix cores leave the kernel memory-bound.
template <bool STATS>
__global__ __launch_bounds__(256, 4) void conv1_fwd_row_kernel(const float* __restrict__ X, const float* __restrict__ Wt,
                                                            bf16* __restrict__ Y, float* __restrict__ part, int N,
                                                            int IH, int IW, int OH, int OW) {
  constexpr int IWM = 320;
  __shared__ __attribute__((aligned(16))) float sx[9 * IWM];   // [9 rows][P]
  __shared__ __attribute__((aligned(16))) unsigned so[W1R_OWM * 16];   // the output row [OW][32] bf16
  __shared__ float red[2][4][C1];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, l16 = lane & 15, kq = lane >> 4;
  const int P = pitch1(IW), T = N * OH;
  const long fsz = (long)IH * IW;
  const XRowChunks xm = xrow_chunks(tid, IH, IW, P);
  // B fragments: kernel rows co = 16 cb + l16, taps k = 8 kq .. 8 kq + 7 (zero past 27); A gather offsets
  // of this lane's taps inside the staged rows: tap k = 3 r + kx reads row r at column 2 p + kx
  bf16x8 wb[2], wl[2];   // kernel head / tail
  int toff[8];
  unsigned kok = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int k = 8 * kq + i;
    const bool ok = k < K1;
    toff[i] = ok ? (k / 3) * P + k % 3 : 0;
    kok |= ok ? 1u << i : 0u;
#pragma unroll
    for (int cb = 0; cb < 2; ++cb) {
      const float wv = ok ? Wt[(16 * cb + l16) * K1 + k] : 0.f;
      wb[cb][i] = (bf16)wv;
      wl[cb][i] = (bf16)(wv - (float)wb[cb][i]);
    }
  }
  f4a4 rx[3];
  auto fetch = [&](int t) {
    const int n = t / OH, oh = t - n * OH;
    xrow_fetch(X + (long)n * 3 * fsz + (long)(2 * oh) * IW, xm, rx);
  };
  float s1[2] = {0.f, 0.f}, s2[2] = {0.f, 0.f};
  bf16* sob = reinterpret_cast<bf16*>(so);
  typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
  const int npg = (OW + 15) / 16;
  fetch(blockIdx.x);   // (the grid never exceeds the tile count)
  for (int t = blockIdx.x; t < T; t += gridDim.x) {
    __syncthreads();   // the previous tile's LDS reads (input rows, output row) are done
    xrow_store(sx, xm, rx);
    __syncthreads();
    fetch(min(t + (int)gridDim.x, T - 1));
    for (int g = w; g < npg; g += 4) {
      const int pa = min(g * 16 + l16, OW - 1);   // A row (clamped: rows past OW are not stored)
      float xv[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) xv[i] = sx[toff[i] + 2 * pa];
      bf16x8 a, al;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const float v = ((kok >> i) & 1) ? xv[i] : 0.f;
        a[i] = (bf16)v;
        al[i] = (bf16)(v - (float)a[i]);
      }
      const f32x4 z = f32x4{0.f, 0.f, 0.f, 0.f};
      f32x4 acc[2];
#pragma unroll
      for (int cb = 0; cb < 2; ++cb) {
        acc[cb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al, wb[cb], z, 0, 0, 0);          // small terms first
        acc[cb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, wl[cb], acc[cb], 0, 0, 0);
        acc[cb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, wb[cb], acc[cb], 0, 0, 0);
      }
      // acc[cb][r] = y[pixel 16 g + 4 kq + r][channel 16 cb + l16]
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int p = g * 16 + 4 * kq + r;
        if (p < OW) {
#pragma unroll
          for (int cb = 0; cb < 2; ++cb) {
            const bf16 ob = (bf16)acc[cb][r];
            sob[p * C1 + 16 * cb + l16] = ob;
            if constexpr (STATS) {
              const float q = (float)ob;
              s1[cb] += q;
              s2[cb] = fmaf(q, q, s2[cb]);
            }
          }
        }
      }
    }
    __syncthreads();   // the output row is staged: 16-B stores, 4 lanes per pixel
    u32x4* yrow = reinterpret_cast<u32x4*>(Y + (long)t * OW * C1);
    const u32x4* so4 = reinterpret_cast<const u32x4*>(so);
#pragma unroll
    for (int k = 0; k < W1R_DL; ++k)
      if (tid + 256 * k < OW * 4) yrow[tid + 256 * k] = so4[tid + 256 * k];
  }
  if constexpr (STATS) {
#pragma unroll
    for (int cb = 0; cb < 2; ++cb) {
      float a = s1[cb], b = s2[cb];
      a += __shfl_xor(a, 16, 64);
      a += __shfl_xor(a, 32, 64);
      b += __shfl_xor(b, 16, 64);
      b += __shfl_xor(b, 32, 64);
      if (lane < 16) {
        red[0][w][16 * cb + l16] = a;
        red[1][w][16 * cb + l16] = b;
      }
    }
    __syncthreads();
    if (tid < 2 * C1) {
      const int st = tid >> 5, c = tid & 31;
      part[((long)blockIdx.x * 2 + st) * C1 + c] = (red[st][0][c] + red[st][1][c]) + (red[st][2][c] + red[st][3][c]);
    }
  }
}

// Weight gradient over one output row per tile (bf16 output gradients, frames up to W1R_IW wide), with
// the next tile's operands prefetched into registers while the current tile is computed from LDS, and
// (MODE 1 / 2) BN1's backward apply fused into the load of the output gradient:
//   dC1[p][c] = bf16(alpha[c] * g + bcoef[c] * y + delta[c]),  g = dZ[p][c], masked to 0 where
//   y * ms[c] + mt[c] <= 0 (MODE 2: dZ is the gradient of relu(bn1(y)), Xception.py:170)
// -- the value bn_bwd_apply_kernel stores (same fma order, same bf16 rounding), so the fused path equals
// xcp_bn_bwd_apply + xcp_conv1_wgrad on the stored tensor bit for bit.  MODE 0: dZ is dC1 itself.
// Per tile: the three stride-2 input rows of each input channel (fp32, 16-B loads) and the output row of
// dZ (and y) (16-B loads), ~31 KB.  The sum over pixels runs on the matrix cores: per 32 pixels and
// wave, dW[32 co][32 taps] += dC1^T[32 co][32 px] x Xcol[32 px][32 taps] as v_mfma_f32_16x16x32_bf16
// (dC1 -- bf16 already -- read by transposed LDS reads, ds_read_b64_tr_b16, and formed on the spot; the
// gathered inputs split into a bf16 head and tail, two MFMAs per block, so the products are exact to
// ~2^-17 as in the forward; fp32 accumulation).  No LDS-DMA (a plain LDS read after one makes hipcc drain every outstanding load), so
// the prefetch stays in flight through the compute.
template <int MODE>
__global__ __launch_bounds__(256, 3) void conv1_wgrad_row_kernel(const float* __restrict__ X, const bf16* __restrict__ dZ,
                                                              const bf16* __restrict__ Yv, const float* alpha,
                                                              const float* bcoef, const float* delta, const float* ms,
                                                              const float* mt, float* __restrict__ part, int N, int IH,
                                                              int IW, int OH, int OW) {
  constexpr bool BN = MODE != 0;
  constexpr int RPX = W1R_OW + 1;   // staged pixels per row (one spare: the transposed reads of the last
                                    // 32-pixel group may address pixel OW)
  __shared__ __attribute__((aligned(16))) char smem[9 * W1R_IW * 4 + 2 * RPX * 64];
  float* sx = reinterpret_cast<float*>(smem);                                    // [9 rows][P]
  typedef unsigned u32x4 __attribute__((ext_vector_type(4)));   // (HIP's uint4 struct arrays end up in scratch)
  u32x4* sd = reinterpret_cast<u32x4*>(smem + 9 * W1R_IW * 4);                   // [OW * 4] chunks of dZ
  u32x4* sy = sd + RPX * 4;                                                      // [OW * 4] chunks of y
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, l16 = lane & 15, kq = lane >> 4;
  const int P = pitch1(IW), nch = OW * 4, T = N * OH;
  const long fsz = (long)IH * IW;
  const XRowChunks xm = xrow_chunks(tid, IH, IW, P);
  // this lane's channels 16 cb + l16 (A rows) and their coefficients; its taps 16 kb + l16 (B columns)
  float al[2] = {1.f, 1.f}, bc[2] = {0.f, 0.f}, de[2] = {0.f, 0.f}, sm[2] = {1.f, 1.f}, tm[2] = {0.f, 0.f};
  int boff[2];
  bool bok[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int c = 16 * h + l16;
    if constexpr (BN) {
      al[h] = alpha[c];
      bc[h] = bcoef[c];
      de[h] = delta[c];
    }
    if constexpr (MODE == 2) {
      sm[h] = ms[c];
      tm[h] = mt[c];
    }
    const int k = 16 * h + l16;
    bok[h] = k < K1;
    boff[h] = bok[h] ? (k / 3) * P + k % 3 : 0;
  }
  f4a4 rx[3];
  u32x4 rd[W1R_DL], ry[BN ? W1R_DL : 1];
  // operands of tile t (always a valid tile: loads are unconditional, from clamped addresses)
  auto fetch = [&](int t) {
    const int n = t / OH, oh = t - n * OH;
    xrow_fetch(X + (long)n * 3 * fsz + (long)(2 * oh) * IW, xm, rx);
    const long db = ((long)n * OH + oh) * OW * C1;
#pragma unroll
    for (int i = 0; i < W1R_DL; ++i) {
      const int j = min(tid + 256 * i, nch - 1);
      rd[i] = *reinterpret_cast<const u32x4*>(dZ + db + j * 8);
      if constexpr (BN) ry[i] = *reinterpret_cast<const u32x4*>(Yv + db + j * 8);
    }
  };
  f32x4 acc[2][2];   // [co block][tap block]: lane holds dW[16 cb + 4 kq + r][16 kb + l16]
#pragma unroll
  for (int cb = 0; cb < 2; ++cb)
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) acc[cb][kb] = f32x4{0.f, 0.f, 0.f, 0.f};
  const char* sdc = reinterpret_cast<const char*>(sd);
  const char* syc = reinterpret_cast<const char*>(sy);
  const int q = l16 >> 2, pp = l16 & 3;   // transposed read: lane 4q + pp addresses pixel row q, channels 4pp..4pp+3
  const int ngr = (OW + 31) / 32;
  fetch(blockIdx.x);   // (the grid never exceeds the tile count)
  for (int t = blockIdx.x; t < T; t += gridDim.x) {
    __syncthreads();   // the previous tile's LDS reads are done
    xrow_store(sx, xm, rx);
    static_assert(W1R_DL == 3, "the chunk stores below are written out for three chunks per thread");
    auto put = [&](int i, const u32x4& v, const u32x4& wv) {
      if (tid + 256 * i < nch) {
        sd[tid + 256 * i] = v;
        if constexpr (BN) sy[tid + 256 * i] = wv;
      }
    };
    put(0, rd[0], ry[BN ? 0 : 0]);
    put(1, rd[1], ry[BN ? 1 : 0]);
    put(2, rd[2], ry[BN ? 2 : 0]);
    __syncthreads();
    fetch(min(t + (int)gridDim.x, T - 1));   // next tile (the last tile once more past the end)
    for (int g = w; g < ngr; g += 4) {
      const int p0 = 32 * g + 8 * kq;   // this lane's 8 pixels: A columns, B rows
      bf16x8 a[2], b[2], bl[2];
#pragma unroll
      for (int cb = 0; cb < 2; ++cb) {
        const int o0 = ((p0 + q) * C1 + 16 * cb + 4 * pp) * 2, o1 = o0 + 4 * C1 * 2;
        const bf16x4 d0 = ds_read_tr(sdc + o0), d1 = ds_read_tr(sdc + o1);
        bf16x4 y0 = d0, y1 = d1;
        if constexpr (BN) {
          y0 = ds_read_tr(syc + o0);
          y1 = ds_read_tr(syc + o1);
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          float d = (float)(i < 4 ? d0[i] : d1[i - 4]);
          if constexpr (BN) {
            const float y = (float)(i < 4 ? y0[i] : y1[i - 4]);
            if constexpr (MODE == 2) d = fmaf(y, sm[cb], tm[cb]) > 0.f ? d : 0.f;
            d = fmaf(al[cb], d, fmaf(bc[cb], y, de[cb]));
          }
          a[cb][i] = (bf16)(p0 + i < OW ? d : 0.f);
        }
      }
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const int pc = min(p0 + i, OW - 1);
          const float x = bok[kb] && p0 + i < OW ? sx[boff[kb] + 2 * pc] : 0.f;
          b[kb][i] = (bf16)x;
          bl[kb][i] = (bf16)(x - (float)b[kb][i]);
        }
#pragma unroll
      for (int cb = 0; cb < 2; ++cb)
#pragma unroll
        for (int kb = 0; kb < 2; ++kb) {
          acc[cb][kb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[cb], bl[kb], acc[cb][kb], 0, 0, 0);
          acc[cb][kb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[cb], b[kb], acc[cb][kb], 0, 0, 0);
        }
    }
  }
  // reduce the 4 waves in LDS: red[wave][co][tap < 27]
  __syncthreads();
  float* red = reinterpret_cast<float*>(smem);   // [4 waves][C1][K1] (13.8 KB)
#pragma unroll
  for (int cb = 0; cb < 2; ++cb)
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
      if (bok[kb]) {
#pragma unroll
        for (int r = 0; r < 4; ++r) red[(w * C1 + 16 * cb + 4 * kq + r) * K1 + 16 * kb + l16] = acc[cb][kb][r];
      }
  __syncthreads();
  for (int i = tid; i < C1 * K1; i += 256) {
    float v = 0.f;
#pragma unroll
    for (int qq = 0; qq < 4; ++qq) v += red[qq * C1 * K1 + i];
    part[(long)blockIdx.x * (C1 * K1) + i] = v;
  }
}

}  // namespace

namespace {
// The tiled kernels stage input rows in LDS; frames wider than their 64 KB budget (IW > ~690)
// fall back to the per-pixel kernels.
constexpr int F1_TH = 4;
}

extern "C" {

int xcp_conv1_wgrad_fused(int dtype, int IH, int IW);

// partial rows of xcp_conv1_fwd_stats ([parts][2][32]): one per workgroup of the row kernel
int xcp_conv1_fwd_parts(int N, int IH, int IW) {
  const int OH = (IH - 3) / 2 + 1;
  const long tiles = (long)N * OH;
  return (int)(tiles < 1024 ? (tiles > 0 ? tiles : 0) : 1024);
}

int xcp_conv1_fwd(int dtype, const float* X, const float* W, void* Y, int N, int IH, int IW, hipStream_t st) {
  const int OH = (IH - 3) / 2 + 1, OW = (IW - 3) / 2 + 1;
  const long total = (long)N * OH * OW * (C1 / 8);
  if (total <= 0) return XCP_OK;
  if (xcp_conv1_wgrad_fused(dtype, IH, IW)) {
    hipLaunchKernelGGL(conv1_fwd_row_kernel<false>, dim3(xcp_conv1_fwd_parts(N, IH, IW)), dim3(256), 0, st, X, W,
                       (bf16*)Y, nullptr, N, IH, IW, OH, OW);
    return (int)hipGetLastError();
  }
  const size_t lds = ((size_t)3 * (2 * F1_TH + 1) * ((IW + 63) & ~63) + C1 * K1) * sizeof(float);
  if (lds <= 64 * 1024) {
    const unsigned blocks = (unsigned)(N * ((OH + F1_TH - 1) / F1_TH));
    if (dtype == XCP_BF16)
      hipLaunchKernelGGL((conv1_fwd_tile_kernel<bf16, F1_TH>), dim3(blocks), dim3(256), lds, st, X, W, (bf16*)Y, N, IH,
                         IW, OH, OW);
    else if (dtype == XCP_F32)
      hipLaunchKernelGGL((conv1_fwd_tile_kernel<float, F1_TH>), dim3(blocks), dim3(256), lds, st, X, W, (float*)Y, N,
                         IH, IW, OH, OW);
    else
      return XCP_EUNSUPPORTED;
    return (int)hipGetLastError();
  }
  const unsigned g = (unsigned)((total + 255) / 256);
  if (dtype == XCP_BF16)
    hipLaunchKernelGGL(conv1_fwd_kernel<bf16>, dim3(g), dim3(256), 0, st, X, W, (bf16*)Y, N, IH, IW, OH, OW);
  else if (dtype == XCP_F32)
    hipLaunchKernelGGL(conv1_fwd_kernel<float>, dim3(g), dim3(256), 0, st, X, W, (float*)Y, N, IH, IW, OH, OW);
  else
    return XCP_EUNSUPPORTED;
  return (int)hipGetLastError();
}

// number of partial rows xcp_conv1_wgrad writes ([parts][32*27])
static size_t conv1_wgrad_lds(int dtype, int IW, int OW) {
  const size_t in = (size_t)3 * (2 * W1_TH + 1) * ((IW + 63) & ~63) * sizeof(float);
  const size_t dy = (size_t)W1_TH * OW * C1 * (dtype == XCP_BF16 ? 2 : 4);
  const size_t red = (size_t)4 * C1 * K1 * sizeof(float);
  return (in + dy > red ? in + dy : red);
}

int xcp_conv1_wgrad_parts(int N, int IH, int IW) {
  const int OH = (IH - 3) / 2 + 1, OW = (IW - 3) / 2 + 1;
  if (conv1_wgrad_lds(XCP_F32, IW, OW) <= 64 * 1024) {
    const int tiles = N * ((OH + W1_TH - 1) / W1_TH);
    return tiles < 1024 ? tiles : 1024;
  }
  const long P = (long)N * OH * OW;
  long blocks = 1024;
  const long minpix = 64 * 8;
  if (P / blocks < minpix) blocks = (P + minpix - 1) / minpix;
  if (blocks < 1) blocks = 1;
  return (int)blocks;
}

// 1 when the row kernel (and so xcp_conv1_wgrad_bn) takes this shape: bf16, frames <= 320 wide
int xcp_conv1_wgrad_fused(int dtype, int IH, int IW) {
  return dtype == XCP_BF16 && IW >= 3 && IH >= 3 && IW <= W1R_IW && 3L * IH * IW < (1L << 30);
}

int xcp_conv1_wgrad(int dtype, const float* X, const void* dY, float* part, int N, int IH, int IW, hipStream_t st) {
  const int OH = (IH - 3) / 2 + 1, OW = (IW - 3) / 2 + 1;
  const long P = (long)N * OH * OW;
  const int blocks = xcp_conv1_wgrad_parts(N, IH, IW);
  if (P <= 0) return XCP_OK;
  if (xcp_conv1_wgrad_fused(dtype, IH, IW)) {
    hipLaunchKernelGGL(conv1_wgrad_row_kernel<0>, dim3(blocks), dim3(256), 0, st, X, (const bf16*)dY, nullptr, nullptr,
                       nullptr, nullptr, nullptr, nullptr, part, N, IH, IW, OH, OW);
    return (int)hipGetLastError();
  }
  if (conv1_wgrad_lds(XCP_F32, IW, OW) <= 64 * 1024) {
    const size_t lds = conv1_wgrad_lds(dtype, IW, OW);
    if (dtype == XCP_BF16)
      hipLaunchKernelGGL(conv1_wgrad_tile_kernel<bf16>, dim3(blocks), dim3(256), lds, st, X, (const bf16*)dY, part, N, IH,
                         IW, OH, OW);
    else if (dtype == XCP_F32)
      hipLaunchKernelGGL(conv1_wgrad_tile_kernel<float>, dim3(blocks), dim3(256), lds, st, X, (const float*)dY, part, N,
                         IH, IW, OH, OW);
    else
      return XCP_EUNSUPPORTED;
    return (int)hipGetLastError();
  }
  const long ppb = (P + blocks - 1) / blocks;
  if (dtype == XCP_BF16)
    hipLaunchKernelGGL(conv1_wgrad_kernel<bf16>, dim3(blocks), dim3(256), 0, st, X, (const bf16*)dY, part, N, IH, IW, OH,
                       OW, ppb);
  else if (dtype == XCP_F32)
    hipLaunchKernelGGL(conv1_wgrad_kernel<float>, dim3(blocks), dim3(256), 0, st, X, (const float*)dY, part, N, IH, IW,
                       OH, OW, ppb);
  else
    return XCP_EUNSUPPORTED;
  return (int)hipGetLastError();
}

int xcp_permute3(int out_dtype, const float* in, void* out, int d0, int d1, int d2, int p0, int p1, int p2,
                 hipStream_t st) {
  const long total = (long)d0 * d1 * d2;
  if (total <= 0) return XCP_OK;
  if (p0 + p1 + p2 != 3 || p0 == p1 || p1 == p2 || p0 == p2) return XCP_EINVAL;
  const unsigned g = (unsigned)((total + 255) / 256);
  if (out_dtype == XCP_BF16)
    hipLaunchKernelGGL(permute3_kernel<bf16>, dim3(g), dim3(256), 0, st, in, (bf16*)out, d0, d1, d2, p0, p1, p2);
  else if (out_dtype == XCP_F32)
    hipLaunchKernelGGL(permute3_kernel<float>, dim3(g), dim3(256), 0, st, in, (float*)out, d0, d1, d2, p0, p1, p2);
  else
    return XCP_EUNSUPPORTED;
  return (int)hipGetLastError();
}

// workgroups xcp_permute3_batch gives one job (the job table's first-block column advances by it)
int xcp_permute3_blocks(int d0, int d1, int d2, int p0, int p1, int p2, long s0, long s1) {
  const PermPlan q = perm_plan(d0, d1, d2, p0, p1, p2, s0, s1);
  if (q.mode == 2) return (int)(((long)d0 * d1 * d2 + 255) / 256);
  return q.tiles();
}

// njobs permute3 jobs ([njobs][12] int64 on the device, see permute3_batch_kernel) covering
// nblocks workgroups in total; the host validates the permutations when it builds them
int xcp_permute3_batch(const long long* jobs, int njobs, int nblocks, hipStream_t st) {
  if (njobs <= 0 || nblocks <= 0) return XCP_OK;
  hipLaunchKernelGGL(permute3_batch_kernel, dim3(nblocks), dim3(256), 0, st, jobs, njobs);
  return (int)hipGetLastError();
}

// conv1 weight gradient with BN1's backward apply fused into the load of its output gradient (see
// conv1_wgrad_row_kernel): part[blocks][32*27] as xcp_conv1_wgrad on dC1 = alpha*mask(dZ) + bcoef*Y + delta;
// mscale / mshift (BN1's forward scale / shift) null: no ReLU mask.  Shapes: xcp_conv1_wgrad_fused.
int xcp_conv1_wgrad_bn(int dtype, const float* X, const void* dZ, const void* Y, const float* alpha, const float* bcoef,
                       const float* delta, const float* mscale, const float* mshift, float* part, int N, int IH, int IW,
                       hipStream_t st) {
  if (!xcp_conv1_wgrad_fused(dtype, IH, IW)) return XCP_EUNSUPPORTED;
  if ((mscale == nullptr) != (mshift == nullptr)) return XCP_EINVAL;
  const int OH = (IH - 3) / 2 + 1, OW = (IW - 3) / 2 + 1;
  if ((long)N * OH * OW <= 0) return XCP_OK;
  const int blocks = xcp_conv1_wgrad_parts(N, IH, IW);
  if (mscale)
    hipLaunchKernelGGL(conv1_wgrad_row_kernel<2>, dim3(blocks), dim3(256), 0, st, X, (const bf16*)dZ, (const bf16*)Y,
                       alpha, bcoef, delta, mscale, mshift, part, N, IH, IW, OH, OW);
  else
    hipLaunchKernelGGL(conv1_wgrad_row_kernel<1>, dim3(blocks), dim3(256), 0, st, X, (const bf16*)dZ, (const bf16*)Y,
                       alpha, bcoef, delta, nullptr, nullptr, part, N, IH, IW, OH, OW);
  return (int)hipGetLastError();
}

// conv1 forward (bf16 output) with BN1's batch-statistics partials part[xcp_conv1_fwd_parts][2][32]
// (sum y, sum y^2 over the stored outputs), shapes as xcp_conv1_wgrad_fused
int xcp_conv1_fwd_stats(int dtype, const float* X, const float* W, void* Y, float* part, int N, int IH, int IW,
                        hipStream_t st) {
  if (!xcp_conv1_wgrad_fused(dtype, IH, IW)) return XCP_EUNSUPPORTED;
  const int OH = (IH - 3) / 2 + 1, OW = (IW - 3) / 2 + 1;
  if ((long)N * OH * OW <= 0) return XCP_OK;
  hipLaunchKernelGGL(conv1_fwd_row_kernel<true>, dim3(xcp_conv1_fwd_parts(N, IH, IW)), dim3(256), 0, st, X, W, (bf16*)Y,
                     part, N, IH, IW, OH, OW);
  return (int)hipGetLastError();
}

}  // extern "C"
