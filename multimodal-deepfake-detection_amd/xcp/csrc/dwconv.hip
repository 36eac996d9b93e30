// Depthwise 3x3 convolution (stride 1, pad 1, no bias), NHWC, forward and fused
// backward (dgrad + wgrad + activation mask + residual / skip-gradient adds).
//
// Reference op: SeparableConv2d.conv1 = nn.Conv2d(C, C, 3, 1, 1, groups=C,
// bias=False) (Xception.py:41, called at :45), always preceded in the
// backbone by a ReLU and usually by the previous BatchNorm (Block.rep,
// Xception.py:61-87).  That input transform is applied on load:
//   ACT_NONE   : a = x                         (block1's first rep, Xception.py:80-81)
//   ACT_RELU   : a = max(x, 0)                 (first rep of blocks 2-12, :83)
//   ACT_BNRELU : a = max(x*scale[c]+shift[c],0) (BN of the previous rep + ReLU)
// HBM-bound: every thread owns CPT channels of a strip of R output pixels along
// W and slides a 3x3 register window, so each input vector is fetched ~once.
#include "common.h"

namespace {

template <int ACT, int CPT>
XCP_DEV void act_apply(float* v, const float* sc, const float* sh) {
  if constexpr (ACT == ACT_RELU) {
#pragma unroll
    for (int j = 0; j < CPT; ++j) v[j] = fmaxf(v[j], 0.f);
  } else if constexpr (ACT == ACT_BNRELU) {
#pragma unroll
    for (int j = 0; j < CPT; ++j) v[j] = fmaxf(fmaf(v[j], sc[j], sh[j]), 0.f);
  }
}

struct DwArgs {
  const void* X;        // [N,H,W,C] raw input (pre-transform)
  void* Y;              // [N,H,W,C] output
  const float* Wt;      // [9][C] taps (tap = ky*3+kx)
  const float* scale;   // [C] (ACT_BNRELU)
  const float* shift;   // [C]
  int N, H, W, C, R, nstrips;
};

template <typename T, int ACT, int CPT>
__global__ __launch_bounds__(256) void dw_fwd_kernel(DwArgs a) {
  const int CV = a.C / CPT;
  const long g = (long)blockIdx.x * 256 + threadIdx.x;
  const int cv = (int)(g % CV);
  const long u = g / CV;
  const int strip = (int)(u % a.nstrips);
  const long row = u / a.nstrips;   // n*H + h
  if (row >= (long)a.N * a.H) return;
  const int h = (int)(row % a.H);
  const long nbase = (row - h) * a.W;   // pixel index of (n, 0, 0)
  const int c0 = cv * CPT;
  const int w0 = strip * a.R, w1 = min(a.W, w0 + a.R);
  const T* X = reinterpret_cast<const T*>(a.X);
  T* Y = reinterpret_cast<T*>(a.Y);

  float wt[9][CPT], sc[CPT], sh[CPT];
#pragma unroll
  for (int t = 0; t < 9; ++t) VecIO<float, CPT>::load(a.Wt + (long)t * a.C + c0, wt[t]);
  if constexpr (ACT == ACT_BNRELU) {
    VecIO<float, CPT>::load(a.scale + c0, sc);
    VecIO<float, CPT>::load(a.shift + c0, sh);
  }
  auto ld = [&](int hh, int ww, float* v) {
    if (hh < 0 || hh >= a.H || ww < 0 || ww >= a.W) {
#pragma unroll
      for (int j = 0; j < CPT; ++j) v[j] = 0.f;
      return;
    }
    VecIO<T, CPT>::load(X + (nbase + (long)hh * a.W + ww) * a.C + c0, v);
    act_apply<ACT, CPT>(v, sc, sh);
  };
  float win[3][3][CPT];   // [ky][col: w-1,w,w+1][ch]
#pragma unroll
  for (int ky = 0; ky < 3; ++ky) {
    ld(h + ky - 1, w0 - 1, win[ky][0]);
    ld(h + ky - 1, w0, win[ky][1]);
  }
  for (int w = w0; w < w1; ++w) {
#pragma unroll
    for (int ky = 0; ky < 3; ++ky) ld(h + ky - 1, w + 1, win[ky][2]);
    float o[CPT];
#pragma unroll
    for (int j = 0; j < CPT; ++j) {
      float s = 0.f;
#pragma unroll
      for (int ky = 0; ky < 3; ++ky)
#pragma unroll
        for (int kx = 0; kx < 3; ++kx) s = fmaf(win[ky][kx][j], wt[ky * 3 + kx][j], s);
      o[j] = s;
    }
    VecIO<T, CPT>::store(Y + (nbase + (long)h * a.W + w) * a.C + c0, o);
#pragma unroll
    for (int ky = 0; ky < 3; ++ky)
#pragma unroll
      for (int j = 0; j < CPT; ++j) {
        win[ky][0][j] = win[ky][1][j];
        win[ky][1][j] = win[ky][2][j];
      }
  }
}

// ---------------------------------------------------------------------------------
// Fused backward.  Per output-gradient pixel p:
//   dA[p]   = sum_tap dY[p - off(tap)] * w[tap]          (transposed 3x3)
//   dX[p]   = act'(p) * dA[p] + dRes[p] + (p at even (h,w) ? dSkip[p/2] : 0)
//   dW[tap] += dY[p] * a[p + off(tap)]                   (block partial -> slab)
// act'(p) = (a[p] > 0) for ACT_RELU / ACT_BNRELU (gradient w.r.t. the BN output
// for ACT_BNRELU), 1 for ACT_NONE.
struct DwBwdArgs {
  const void* dY;       // [N,H,W,C] gradient of the depthwise output
  const void* X;        // [N,H,W,C] raw depthwise input (pre-transform)
  const float* Wt;      // [9][C]
  const float* scale;
  const float* shift;
  const void* dRes;     // [N,H,W,C] or null (identity-skip gradient)
  const void* dSkip;    // [N,OH,OW,C] or null (stride-2 skip-conv input gradient)
  int sOH, sOW, sS;
  void* dX;             // [N,H,W,C] out
  float* dWpart;        // [P][C][9] per-block-row partials
  int N, H, W, C, R, nstrips;
  int CVB, SPB;         // channel-vectors per block, strip slots per block
  long strips_per_chunk;
};

template <typename T, int ACT, int CPT>
__global__ __launch_bounds__(256) void dw_bwd_kernel(DwBwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) float red[];   // [SPB][CVB*CPT*9]
  const int CV = a.C / CPT;
  const int nchunks = (CV + a.CVB - 1) / a.CVB;
  const int cchunk = blockIdx.x % nchunks;
  const int pchunk = blockIdx.x / nchunks;
  const int tid = threadIdx.x;
  const int lcv = tid % a.CVB, slot = tid / a.CVB;
  const int cv = cchunk * a.CVB + lcv;
  const bool active = slot < a.SPB && cv < CV;
  const int c0 = cv * CPT;
  const T* dY = reinterpret_cast<const T*>(a.dY);
  const T* X = reinterpret_cast<const T*>(a.X);
  const T* dRes = reinterpret_cast<const T*>(a.dRes);
  const T* dSkip = reinterpret_cast<const T*>(a.dSkip);
  T* dX = reinterpret_cast<T*>(a.dX);

  float wt[9][CPT], sc[CPT], sh[CPT], dw[9][CPT];
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int j = 0; j < CPT; ++j) dw[t][j] = 0.f;
  if (active) {
#pragma unroll
    for (int t = 0; t < 9; ++t) VecIO<float, CPT>::load(a.Wt + (long)t * a.C + c0, wt[t]);
    if constexpr (ACT == ACT_BNRELU) {
      VecIO<float, CPT>::load(a.scale + c0, sc);
      VecIO<float, CPT>::load(a.shift + c0, sh);
    }
    const long total = (long)a.N * a.H * a.nstrips;
    const long sbeg = (long)pchunk * a.strips_per_chunk;
    const long send = min(total, sbeg + a.strips_per_chunk);
    for (long su = sbeg + slot; su < send; su += a.SPB) {
      const int strip = (int)(su % a.nstrips);
      const long row = su / a.nstrips;
      const int h = (int)(row % a.H);
      const int n = (int)(row / a.H);
      const long nbase = (long)n * a.H * a.W;
      const int w0 = strip * a.R, w1 = min(a.W, w0 + a.R);
      auto ldx = [&](int hh, int ww, float* v) {
        if (hh < 0 || hh >= a.H || ww < 0 || ww >= a.W) {
#pragma unroll
          for (int j = 0; j < CPT; ++j) v[j] = 0.f;
          return;
        }
        VecIO<T, CPT>::load(X + (nbase + (long)hh * a.W + ww) * a.C + c0, v);
        act_apply<ACT, CPT>(v, sc, sh);
      };
      auto ldg = [&](int hh, int ww, float* v) {
        if (hh < 0 || hh >= a.H || ww < 0 || ww >= a.W) {
#pragma unroll
          for (int j = 0; j < CPT; ++j) v[j] = 0.f;
          return;
        }
        VecIO<T, CPT>::load(dY + (nbase + (long)hh * a.W + ww) * a.C + c0, v);
      };
      float xa[3][3][CPT], gy[3][3][CPT];
#pragma unroll
      for (int ky = 0; ky < 3; ++ky) {
        ldx(h + ky - 1, w0 - 1, xa[ky][0]);
        ldx(h + ky - 1, w0, xa[ky][1]);
        ldg(h + ky - 1, w0 - 1, gy[ky][0]);
        ldg(h + ky - 1, w0, gy[ky][1]);
      }
      for (int w = w0; w < w1; ++w) {
#pragma unroll
        for (int ky = 0; ky < 3; ++ky) {
          ldx(h + ky - 1, w + 1, xa[ky][2]);
          ldg(h + ky - 1, w + 1, gy[ky][2]);
        }
        float o[CPT];
#pragma unroll
        for (int j = 0; j < CPT; ++j) {
          // dgrad: input pixel p receives dY[p - off] * w[off]; off = (ky-1, kx-1)
          float s = 0.f;
#pragma unroll
          for (int ky = 0; ky < 3; ++ky)
#pragma unroll
            for (int kx = 0; kx < 3; ++kx) s = fmaf(gy[2 - ky][2 - kx][j], wt[ky * 3 + kx][j], s);
          // wgrad: dY[p] * a[p + off]
          const float gc = gy[1][1][j];
#pragma unroll
          for (int ky = 0; ky < 3; ++ky)
#pragma unroll
            for (int kx = 0; kx < 3; ++kx) dw[ky * 3 + kx][j] = fmaf(gc, xa[ky][kx][j], dw[ky * 3 + kx][j]);
          if constexpr (ACT != ACT_NONE) s = xa[1][1][j] > 0.f ? s : 0.f;
          o[j] = s;
        }
        const long pix = nbase + (long)h * a.W + w;
        if (dRes) {
          float r[CPT];
          VecIO<T, CPT>::load(dRes + pix * a.C + c0, r);
#pragma unroll
          for (int j = 0; j < CPT; ++j) o[j] += r[j];
        }
        if (dSkip && (h % a.sS) == 0 && (w % a.sS) == 0) {
          const int oh = h / a.sS, ow = w / a.sS;
          if (oh < a.sOH && ow < a.sOW) {
            float r[CPT];
            VecIO<T, CPT>::load(dSkip + (((long)n * a.sOH + oh) * a.sOW + ow) * a.C + c0, r);
#pragma unroll
            for (int j = 0; j < CPT; ++j) o[j] += r[j];
          }
        }
        VecIO<T, CPT>::store(dX + pix * a.C + c0, o);
#pragma unroll
        for (int ky = 0; ky < 3; ++ky)
#pragma unroll
          for (int j = 0; j < CPT; ++j) {
            xa[ky][0][j] = xa[ky][1][j];
            xa[ky][1][j] = xa[ky][2][j];
            gy[ky][0][j] = gy[ky][1][j];
            gy[ky][1][j] = gy[ky][2][j];
          }
      }
    }
  }
  // block reduction of dw over strip slots
  const int L = a.CVB * CPT * 9;
  if (slot < a.SPB) {
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
      for (int j = 0; j < CPT; ++j) red[slot * L + (lcv * CPT + j) * 9 + t] = dw[t][j];
  }
  __syncthreads();
  for (int i = tid; i < L; i += 256) {
    float s = 0.f;
    for (int q = 0; q < a.SPB; ++q) s += red[q * L + i];
    const int c = cchunk * a.CVB * CPT + i / 9;
    if (c < a.C) a.dWpart[((long)pchunk * a.C + c) * 9 + (i % 9)] = s;
  }
}

template <typename T>
int launch_fwd(int act, const DwArgs& a, hipStream_t st) {
  constexpr int CPT = 8;
  const long work = (long)a.N * a.H * a.nstrips * (a.C / CPT);
  const dim3 grid((unsigned)((work + 255) / 256));
  if (act == ACT_NONE) hipLaunchKernelGGL((dw_fwd_kernel<T, ACT_NONE, CPT>), grid, dim3(256), 0, st, a);
  else if (act == ACT_RELU) hipLaunchKernelGGL((dw_fwd_kernel<T, ACT_RELU, CPT>), grid, dim3(256), 0, st, a);
  else hipLaunchKernelGGL((dw_fwd_kernel<T, ACT_BNRELU, CPT>), grid, dim3(256), 0, st, a);
  return (int)hipGetLastError();
}

template <typename T>
int launch_bwd(int act, const DwBwdArgs& a, int nblocks, hipStream_t st) {
  constexpr int CPT = 4;
  const size_t smem = (size_t)a.SPB * a.CVB * CPT * 9 * sizeof(float);
  if (act == ACT_NONE) hipLaunchKernelGGL((dw_bwd_kernel<T, ACT_NONE, CPT>), dim3(nblocks), dim3(256), smem, st, a);
  else if (act == ACT_RELU) hipLaunchKernelGGL((dw_bwd_kernel<T, ACT_RELU, CPT>), dim3(nblocks), dim3(256), smem, st, a);
  else hipLaunchKernelGGL((dw_bwd_kernel<T, ACT_BNRELU, CPT>), dim3(nblocks), dim3(256), smem, st, a);
  return (int)hipGetLastError();
}

int strip_len(int W) {
  const int ns = (W + 7) / 8;
  return (W + ns - 1) / ns;
}

}  // namespace

extern "C" {

int xcp_dw_fwd(int dtype, int act, const void* X, void* Y, const float* Wt, const float* scale, const float* shift, int N,
               int H, int W, int C, hipStream_t stream) {
  if (C % 8) return XCP_EINVAL;
  if (N <= 0 || H <= 0 || W <= 0) return XCP_OK;
  DwArgs a{X, Y, Wt, scale, shift, N, H, W, C, 0, 0};
  a.R = strip_len(W);
  a.nstrips = (W + a.R - 1) / a.R;
  if (dtype == XCP_BF16) return launch_fwd<bf16>(act, a, stream);
  if (dtype == XCP_F32) return launch_fwd<float>(act, a, stream);
  return XCP_EUNSUPPORTED;
}

// number of pixel chunks the backward uses (size of the dWpart slab: [P][C][9])
int xcp_dw_bwd_chunks(int N, int H, int W, int C) {
  const int R = strip_len(W);
  const long strips = (long)N * H * ((W + R - 1) / R);
  const int CV = C / 4;
  const int CVB = (CV + ((CV + 63) / 64) - 1) / ((CV + 63) / 64);
  const int SPB = 256 / CVB;
  const int nch = (CV + CVB - 1) / CVB;
  // aim for ~2048 blocks, each thread handling >= 2 strips
  long P = 2048 / nch;
  if (P < 1) P = 1;
  const long maxP = (strips + 2L * SPB - 1) / (2L * SPB);
  if (P > maxP) P = maxP;
  if (P < 1) P = 1;
  return (int)P;
}

int xcp_dw_bwd(int dtype, int act, const void* dY, const void* X, const float* Wt, const float* scale, const float* shift,
               const void* dRes, const void* dSkip, int sOH, int sOW, int sS, void* dX, float* dWpart, int N, int H, int W,
               int C, hipStream_t stream) {
  if (C % 8) return XCP_EINVAL;
  if (N <= 0 || H <= 0 || W <= 0) return XCP_OK;
  DwBwdArgs a{};
  a.dY = dY; a.X = X; a.Wt = Wt; a.scale = scale; a.shift = shift; a.dRes = dRes; a.dSkip = dSkip;
  a.sOH = sOH; a.sOW = sOW; a.sS = sS > 0 ? sS : 1; a.dX = dX; a.dWpart = dWpart;
  a.N = N; a.H = H; a.W = W; a.C = C;
  a.R = strip_len(W);
  a.nstrips = (W + a.R - 1) / a.R;
  const int CV = C / 4;
  const int nch = (CV + 63) / 64;
  a.CVB = (CV + nch - 1) / nch;
  a.SPB = 256 / a.CVB;
  const int P = xcp_dw_bwd_chunks(N, H, W, C);
  const long strips = (long)N * H * a.nstrips;
  a.strips_per_chunk = (strips + P - 1) / P;
  const int nblocks = P * nch;
  if (dtype == XCP_BF16) return launch_bwd<bf16>(act, a, nblocks, stream);
  if (dtype == XCP_F32) return launch_bwd<float>(act, a, nblocks, stream);
  return XCP_EUNSUPPORTED;
}

}  // extern "C"
