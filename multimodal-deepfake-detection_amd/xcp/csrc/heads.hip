// Classification heads and losses of the training scripts, forward and backward:
//   ArcFaceHead  (train_visual.py:455-474, m = 0.5; train_au_face.py:423-442, m = 0.30)
//       x_n = x / max(|x|, 1e-12), W_n = W / max(|W|, 1e-12) (F.normalize), cos = x_n W_n^T,
//       logits = s * cos, except at the label: s * cos(acos(clamp(cos, -1+1e-7, 1-1e-7)) + m)
//   CBFocalLoss  (train_au_face.py:445-458) and plain cross entropy (gamma = 0, no weights):
//       ce_i = w[y_i] * (logsumexp(z_i) - z_i[y_i]), pt = exp(-ce), loss = mean((1-pt)^gamma ce)
// The heads are tiny (B x C x D with C = 2, D = 128): one wave per row, a single workgroup
// for the parameter gradient so it is reduced deterministically in LDS.  fp32 throughout.
#include "common.h"

namespace {

constexpr float NORM_EPS = 1e-12f;                 // F.normalize default eps
constexpr float CLAMP_LO = -1.f + 1e-7f, CLAMP_HI = 1.f - 1e-7f;   // the clamp bounds, as fp32 scalars
constexpr int HEAD_MAXC = 16;

XCP_DEV float wsum(float v) { return wave_sum(v); }

// norms of the C class rows of W (one wave each), into LDS wn[C]
XCP_DEV void class_norms(const float* W, int C, int D, float* wn) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  for (int j = w; j < C; j += nw) {
    float s = 0.f;
    for (int k = lane; k < D; k += 64) s = fmaf(W[(long)j * D + k], W[(long)j * D + k], s);
    s = wsum(s);
    if (lane == 0) wn[j] = fmaxf(sqrtf(s), NORM_EPS);
  }
}

// cos_ij of row i for every class j (wave-wide, result in every lane); returns max(|x_i|, eps)
XCP_DEV float row_cos(const float* x, const float* W, const float* wn, int C, int D, float* c) {
  const int lane = threadIdx.x & 63;
  float nx = 0.f;
  float dot[HEAD_MAXC];
#pragma unroll
  for (int j = 0; j < HEAD_MAXC; ++j) dot[j] = 0.f;
  for (int k = lane; k < D; k += 64) {
    const float xv = x[k];
    nx = fmaf(xv, xv, nx);
#pragma unroll
    for (int j = 0; j < HEAD_MAXC; ++j)
      if (j < C) dot[j] = fmaf(xv, W[(long)j * D + k], dot[j]);
  }
  nx = fmaxf(sqrtf(wsum(nx)), NORM_EPS);
#pragma unroll
  for (int j = 0; j < HEAD_MAXC; ++j)
    if (j < C) c[j] = wsum(dot[j]) / (nx * wn[j]);
  return nx;
}

__global__ __launch_bounds__(256) void arcface_fwd_kernel(const float* __restrict__ X, const float* __restrict__ W,
                                                          const long long* __restrict__ labels, float* __restrict__ out,
                                                          int B, int C, int D, float s, float m) {
  __shared__ float wn[HEAD_MAXC];
  class_norms(W, C, D, wn);
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= B) return;
  float c[HEAD_MAXC];
  row_cos(X + (long)row * D, W, wn, C, D, c);
  if (lane < C) {
    float v = 0.f;
#pragma unroll
    for (int j = 0; j < HEAD_MAXC; ++j)
      if (j == lane) v = c[j];
    if (labels && labels[row] == lane) {
      const float cc = fminf(fmaxf(v, CLAMP_LO), CLAMP_HI);
      v = cosf(acosf(cc) + m);
    }
    out[(long)row * C + lane] = s * v;
  }
}

// One workgroup: dX row by row (wave per row), dW reduced over the rows in LDS.
__global__ __launch_bounds__(1024) void arcface_bwd_kernel(const float* __restrict__ X, const float* __restrict__ W,
                                                           const long long* __restrict__ labels,
                                                           const float* __restrict__ dout, float* __restrict__ dX,
                                                           float* __restrict__ dW, int B, int C, int D, float s, float m) {
  extern __shared__ float sm[];                 // wn[16] | dWn partials [nw][C][D]
  float* wn = sm;
  float* part = sm + HEAD_MAXC;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  class_norms(W, C, D, wn);
  for (int i = threadIdx.x; i < nw * C * D; i += blockDim.x) part[i] = 0.f;
  __syncthreads();
  float* mine = part + (long)w * C * D;
  for (int row = w; row < B; row += nw) {
    const float* x = X + (long)row * D;
    float c[HEAD_MAXC], gc[HEAD_MAXC];
    const float nx = row_cos(x, W, wn, C, D, c);
    const long long y = labels ? labels[row] : -1;
#pragma unroll
    for (int j = 0; j < HEAD_MAXC; ++j) {
      if (j >= C) break;
      float g = dout[(long)row * C + j] * s;
      if (j == y) {   // d/dc cos(acos(clamp(c)) + m) = sin(theta + m) / sqrt(1 - cc^2) inside the clamp, else 0
        const bool in = c[j] >= CLAMP_LO && c[j] <= CLAMP_HI;
        const float cc = fminf(fmaxf(c[j], CLAMP_LO), CLAMP_HI);
        g = in ? g * sinf(acosf(cc) + m) / sqrtf(1.f - cc * cc) : 0.f;
      }
      gc[j] = g;
    }
    // d x_n = sum_j gc_j W_n[j];  x_n . d x_n for the normalize backward; dW_n[j] += gc_j x_n
    float xnd = 0.f;
    for (int k = lane; k < D; k += 64) {
      const float xn = x[k] / nx;
      float d = 0.f;
#pragma unroll
      for (int j = 0; j < HEAD_MAXC; ++j) {
        if (j >= C) break;
        d = fmaf(gc[j], W[(long)j * D + k] / wn[j], d);
        mine[j * D + k] = fmaf(gc[j], xn, mine[j * D + k]);
      }
      xnd = fmaf(xn, d, xnd);
    }
    xnd = wsum(xnd);
    const bool big = nx > NORM_EPS;   // F.normalize backward: (d - x_n (x_n . d)) / |x| (or d / eps at the clamp)
    for (int k = lane; k < D; k += 64) {
      const float xn = x[k] / nx;
      float d = 0.f;
#pragma unroll
      for (int j = 0; j < HEAD_MAXC; ++j) {
        if (j >= C) break;
        d = fmaf(gc[j], W[(long)j * D + k] / wn[j], d);
      }
      dX[(long)row * D + k] = big ? (d - xn * xnd) / nx : d / NORM_EPS;
    }
  }
  __syncthreads();
  // fold the per-wave partials into wave 0's, then normalize backward per class row (wave j)
  for (int i = threadIdx.x; i < C * D; i += blockDim.x) {
    float t = 0.f;
    for (int q = 0; q < nw; ++q) t += part[(long)q * C * D + i];
    part[i] = t;
  }
  __syncthreads();
  for (int j = w; j < C; j += nw) {
    float t = 0.f;
    for (int k = lane; k < D; k += 64) t = fmaf(W[(long)j * D + k] / wn[j], part[j * D + k], t);
    t = wsum(t);
    const bool big = wn[j] > NORM_EPS;
    for (int k = lane; k < D; k += 64) {
      const float wv = W[(long)j * D + k] / wn[j];
      dW[(long)j * D + k] = big ? (part[j * D + k] - wv * t) / wn[j] : part[j * D + k] / NORM_EPS;
    }
  }
}

// Focal / class-weighted cross entropy, mean over the B rows, one workgroup.  loss (1 float);
// with dZ: dZ = gout * d loss / d z (gout: device scalar, null = 1).
__global__ __launch_bounds__(256) void focal_ce_kernel(const float* __restrict__ Z, const long long* __restrict__ labels,
                                                       const float* __restrict__ wts, float gamma,
                                                       const float* __restrict__ gout, float* __restrict__ loss,
                                                       float* __restrict__ dZ, int B, int C) {
  __shared__ float red[4];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const float go = gout ? gout[0] : 1.f;
  float acc = 0.f;
  for (int row = threadIdx.x; row < B; row += blockDim.x) {
    const float* z = Z + (long)row * C;
    const long long y = labels[row];
    float mx = -INFINITY;
    for (int j = 0; j < C; ++j) mx = fmaxf(mx, z[j]);
    float se = 0.f;
    for (int j = 0; j < C; ++j) se += expf(z[j] - mx);
    const float lse = mx + logf(se);
    const float wy = wts ? wts[y] : 1.f;
    const float ce = wy * (lse - z[y]);
    const float pt = expf(-ce);
    const float om = 1.f - pt;
    const float fw = gamma == 0.f ? 1.f : powf(om, gamma);
    acc += fw * ce;
    if (dZ) {
      // d/dce [(1-pt)^g ce] = g (1-pt)^(g-1) pt ce + (1-pt)^g
      const float dce = (gamma == 0.f ? 1.f : gamma * powf(om, gamma - 1.f) * pt * ce + fw) * go / (float)B;
      for (int j = 0; j < C; ++j) {
        const float p = expf(z[j] - lse);
        dZ[(long)row * C + j] = dce * wy * (p - (j == y ? 1.f : 0.f));
      }
    }
  }
  acc = wave_sum(acc);
  if (lane == 0) red[w] = acc;
  __syncthreads();
  if (threadIdx.x == 0) loss[0] = (red[0] + red[1] + red[2] + red[3]) / (float)B;
}

}  // namespace

extern "C" {

int xcp_arcface_fwd(const float* X, const float* W, const long long* labels, float* out, int B, int C, int D, float s,
                    float m, hipStream_t st) {
  if (B <= 0) return XCP_OK;
  if (C <= 0 || C > HEAD_MAXC || D <= 0) return XCP_EINVAL;
  hipLaunchKernelGGL(arcface_fwd_kernel, dim3((B + 3) / 4), dim3(256), 0, st, X, W, labels, out, B, C, D, s, m);
  return (int)hipGetLastError();
}

int xcp_arcface_bwd(const float* X, const float* W, const long long* labels, const float* dout, float* dX, float* dW,
                    int B, int C, int D, float s, float m, hipStream_t st) {
  if (C <= 0 || C > HEAD_MAXC || D <= 0 || B < 0) return XCP_EINVAL;
  int nw = 16;
  while (nw > 1 && ((size_t)nw * C * D + HEAD_MAXC) * sizeof(float) > 64 * 1024) nw >>= 1;
  if (((size_t)nw * C * D + HEAD_MAXC) * sizeof(float) > 64 * 1024) return XCP_EUNSUPPORTED;
  const size_t smem = ((size_t)nw * C * D + HEAD_MAXC) * sizeof(float);
  hipLaunchKernelGGL(arcface_bwd_kernel, dim3(1), dim3(64 * nw), smem, st, X, W, labels, dout, dX, dW, B, C, D, s, m);
  return (int)hipGetLastError();
}

int xcp_focal_ce(const float* Z, const long long* labels, const float* weights, float gamma, const float* gout,
                 float* loss, float* dZ, int B, int C, hipStream_t st) {
  if (B <= 0 || C <= 0 || gamma < 0.f) return XCP_EINVAL;
  hipLaunchKernelGGL(focal_ce_kernel, dim3(1), dim3(256), 0, st, Z, labels, weights, gamma, gout, loss, dZ, B, C);
  return (int)hipGetLastError();
}

}  // extern "C"
