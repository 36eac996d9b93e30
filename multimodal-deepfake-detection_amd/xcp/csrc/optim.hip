// Fused gradient clipping + Adam over every trainable tensor in two launches.
//
// Reference: train_visual.py:575-577 / train_audio.py:40-44 run
// torch.nn.utils.clip_grad_norm_(params, 1.0) then torch.optim.Adam(lr, weight_decay) (L2 form:
// g += wd * p; m = b1 m + (1 - b1) g; v = b2 v + (1 - b2) g^2; p -= lr / bc1 * m / (sqrt(v) /
// sqrt(bc2) + eps)).  torch runs that as a per-tensor norm pass, a scaling pass and a
// multi-tensor Adam in chunks of launches; here a chunk table ([n][6] int64: param, grad,
// exp_avg, exp_avg_sq, first element, length; lengths <= XCP_OPT_CHUNK) drives
//   xcp_opt_sumsq: per-chunk sum of g^2, then one workgroup turns the partials into the clip
//                  coefficient min(1, max_norm / (||g|| + 1e-6)) and ||g|| in device memory
//                  (no host synchronisation);
//   xcp_opt_adam:  the Adam update with the gradient scaled by that coefficient on the fly.
// HBM-bound: 4 B x (g, p, m, v read + p, m, v written) = 28 B per parameter.
#include "common.h"

namespace {

constexpr int OPT_THREADS = 256;

__global__ __launch_bounds__(OPT_THREADS) void opt_sumsq_kernel(const long long* __restrict__ tab, float* part) {
  const long long* e = tab + (long)blockIdx.x * 6;
  const float* g = reinterpret_cast<const float*>(e[1]) + e[4];
  const int n = (int)e[5];
  float s = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  for (int i = threadIdx.x; i < n; i += 4 * OPT_THREADS) {
    const float a = g[i];
    const float b = i + OPT_THREADS < n ? g[i + OPT_THREADS] : 0.f;
    const float c2 = i + 2 * OPT_THREADS < n ? g[i + 2 * OPT_THREADS] : 0.f;
    const float d = i + 3 * OPT_THREADS < n ? g[i + 3 * OPT_THREADS] : 0.f;
    s = fmaf(a, a, s);
    s1 = fmaf(b, b, s1);
    s2 = fmaf(c2, c2, s2);
    s3 = fmaf(d, d, s3);
  }
  s = (s + s1) + (s2 + s3);
  s = wave_sum(s);
  __shared__ float ws[OPT_THREADS / 64];
  if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = 0.f;
    for (int w = 0; w < OPT_THREADS / 64; ++w) t += ws[w];
    part[blockIdx.x] = t;
  }
}

// out[0] = clip coefficient, out[1] = total norm
__global__ __launch_bounds__(1024) void opt_clipcoef_kernel(const float* __restrict__ part, int n, float max_norm,
                                                            float* out) {
  double s = 0.0;
  for (int i = threadIdx.x; i < n; i += 1024) s += (double)part[i];
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  __shared__ double ws[16];
  if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    double t = 0.0;
    for (int w = 0; w < 16; ++w) t += ws[w];
    const float norm = (float)sqrt(t);
    const float coef = max_norm > 0.f ? fminf(1.f, max_norm / (norm + 1e-6f)) : 1.f;
    out[0] = coef;
    out[1] = norm;
  }
}

__global__ __launch_bounds__(OPT_THREADS) void opt_adam_kernel(const long long* __restrict__ tab,
                                                               const float* __restrict__ coef, float lr, float b1,
                                                               float b2, float eps, float wd, float bc1, float bc2sqrt,
                                                               const float* __restrict__ tdev, double b1d, double b2d) {
  const long long* e = tab + (long)blockIdx.x * 6;
  const long o = e[4];
  float* p = reinterpret_cast<float*>(e[0]) + o;
  const float* g = reinterpret_cast<const float*>(e[1]) + o;
  float* m = reinterpret_cast<float*>(e[2]) + o;
  float* v = reinterpret_cast<float*>(e[3]) + o;
  const int n = (int)e[5];
  const float c = coef ? coef[0] : 1.f;
  if (tdev) {   // step count on the device (graph-captured steps): the host formula, in double
    const double t = (double)tdev[0];
    bc1 = (float)(1.0 - pow(b1d, t));
    bc2sqrt = (float)sqrt(1.0 - pow(b2d, t));
  }
  const float step = lr / bc1;
  // 4 elements per thread per pass, every load issued before the math (memory-level parallelism)
  for (int i0 = threadIdx.x; i0 < n; i0 += 4 * OPT_THREADS) {
    float pv[4], gv[4], mv[4], vv[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int i = min(i0 + u * OPT_THREADS, n - 1);
      pv[u] = p[i];
      gv[u] = g[i];
      mv[u] = m[i];
      vv[u] = v[i];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int i = i0 + u * OPT_THREADS;
      if (i >= n) break;
      float gi = gv[u] * c;
      gi = fmaf(wd, pv[u], gi);
      const float mi = fmaf(b1, mv[u] - gi, gi);               // lerp(m, g, 1 - b1) = g + b1 (m - g)
      const float vi = fmaf(b2, vv[u], (1.f - b2) * gi * gi);
      m[i] = mi;
      v[i] = vi;
      const float denom = sqrtf(vi) / bc2sqrt + eps;
      p[i] = pv[u] - step * mi / denom;
    }
  }
}

}  // namespace

extern "C" {

// part: [nchunks] fp32 scratch; out: [2] fp32 (clip coefficient, total norm); max_norm <= 0: no clip
int xcp_opt_sumsq(const long long* tab, int nchunks, float* part, float max_norm, float* out, hipStream_t st) {
  if (nchunks <= 0) return XCP_OK;
  hipLaunchKernelGGL(opt_sumsq_kernel, dim3(nchunks), dim3(OPT_THREADS), 0, st, tab, part);
  hipLaunchKernelGGL(opt_clipcoef_kernel, dim3(1), dim3(1024), 0, st, part, nchunks, max_norm, out);
  return (int)hipGetLastError();
}

// coef: device clip coefficient (xcp_opt_sumsq's out) or null; bc1 = 1 - b1^t, bc2sqrt = sqrt(1 - b2^t)
int xcp_opt_adam(const long long* tab, int nchunks, const float* coef, float lr, float b1, float b2, float eps, float wd,
                 float bc1, float bc2sqrt, hipStream_t st) {
  if (nchunks <= 0) return XCP_OK;
  hipLaunchKernelGGL(opt_adam_kernel, dim3(nchunks), dim3(OPT_THREADS), 0, st, tab, coef, lr, b1, b2, eps, wd, bc1,
                     bc2sqrt, nullptr, 0.0, 0.0);
  return (int)hipGetLastError();
}

// the same update with the step count read from device memory (tdev[0], the count after this step):
// bc1 = 1 - b1^t, bc2sqrt = sqrt(1 - b2^t) formed on the device in double from the double betas, as
// the host does for xcp_opt_adam -- so a captured (graph-replayed) step needs no host arithmetic
int xcp_opt_adam_dev(const long long* tab, int nchunks, const float* coef, float lr, double b1, double b2, float eps,
                     float wd, const float* tdev, hipStream_t st) {
  if (nchunks <= 0) return XCP_OK;
  if (!tdev) return XCP_EINVAL;
  hipLaunchKernelGGL(opt_adam_kernel, dim3(nchunks), dim3(OPT_THREADS), 0, st, tab, coef, lr, (float)b1, (float)b2, eps,
                     wd, 1.f, 1.f, tdev, b1, b2);
  return (int)hipGetLastError();
}

}  // extern "C"
