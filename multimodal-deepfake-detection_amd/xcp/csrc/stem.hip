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

}  // namespace

extern "C" {

int xcp_conv1_fwd(int dtype, const float* X, const float* W, void* Y, int N, int IH, int IW, hipStream_t st) {
  const int OH = (IH - 3) / 2 + 1, OW = (IW - 3) / 2 + 1;
  const long total = (long)N * OH * OW * (C1 / 8);
  if (total <= 0) return XCP_OK;
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
int xcp_conv1_wgrad_parts(int N, int IH, int IW) {
  const int OH = (IH - 3) / 2 + 1, OW = (IW - 3) / 2 + 1;
  const long P = (long)N * OH * OW;
  long blocks = 1024;
  const long minpix = 64 * 8;
  if (P / blocks < minpix) blocks = (P + minpix - 1) / minpix;
  if (blocks < 1) blocks = 1;
  return (int)blocks;
}

int xcp_conv1_wgrad(int dtype, const float* X, const void* dY, float* part, int N, int IH, int IW, hipStream_t st) {
  const int OH = (IH - 3) / 2 + 1, OW = (IW - 3) / 2 + 1;
  const long P = (long)N * OH * OW;
  const int blocks = xcp_conv1_wgrad_parts(N, IH, IW);
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

}  // extern "C"
