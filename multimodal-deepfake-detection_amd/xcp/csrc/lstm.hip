// Fused single-layer LSTM recurrence (batch_first, gate order i,f,g,o, h0=c0=0),
// forward and backward-through-time, fp32.
//
// Reference op: nn.LSTM(input_size=2048, hidden_size=H, num_layers=1,
// batch_first=True) (XceptionLSTMV.py:18-23, XceptionLSTMA.py:14-19), called at
// XceptionLSTMV.py:67 / XceptionLSTMA.py:56 and directly as
// `model.lstm(features)[0]` in train_visual.py:569.
//
// The input projection x W_ih^T for all T steps is one MFMA GEMM (gemm.hip);
// these kernels run the serial part: one workgroup per clip walks the T steps,
// keeping h in LDS and reading W_hh^T (coalesced across gate lanes) from L2.
#include "common.h"

namespace {

XCP_DEV float sigm(float x) { return 1.f / (1.f + expf(-x)); }

// xproj [B][T][4H] (already x W_ih^T); whhT [H][4H]; bias = b_ih + b_hh added here.
// Outputs: out/h [B][T][H], hprev [B][T][H] (h_{t-1}), c [B][T][H],
// gates [B][T][4H] post-activation (i, f, g, o), h_n / c_n [B][H].
__global__ __launch_bounds__(256) void lstm_fwd_kernel(const float* __restrict__ xproj, const float* __restrict__ whhT,
                                                       const float* __restrict__ bih, const float* __restrict__ bhh,
                                                       float* __restrict__ out, float* __restrict__ hprev,
                                                       float* __restrict__ cst, float* __restrict__ gates,
                                                       float* __restrict__ hn, float* __restrict__ cn, int T, int H) {
  extern __shared__ float sm[];   // h [H], c [H], gate pre-activations [4H]
  float* sh = sm;
  float* sc = sm + H;
  float* sg = sm + 2 * H;
  const int b = blockIdx.x, tid = threadIdx.x;
  const int G4 = 4 * H;
  for (int k = tid; k < H; k += blockDim.x) { sh[k] = 0.f; sc[k] = 0.f; }
  __syncthreads();
  for (int t = 0; t < T; ++t) {
    const float* xp = xproj + ((long)b * T + t) * G4;
    for (int j = tid; j < G4; j += blockDim.x) {
      float acc = xp[j] + bih[j] + bhh[j];
      for (int k = 0; k < H; ++k) acc = fmaf(sh[k], whhT[(long)k * G4 + j], acc);
      sg[j] = acc;
    }
    __syncthreads();
    float* gt = gates + ((long)b * T + t) * G4;
    const long ob = ((long)b * T + t) * H;
    for (int k = tid; k < H; k += blockDim.x) {
      const float ig = sigm(sg[k]), fg = sigm(sg[H + k]), gg = tanhf(sg[2 * H + k]), og = sigm(sg[3 * H + k]);
      const float c = fmaf(fg, sc[k], ig * gg);
      const float h = og * tanhf(c);
      gt[k] = ig; gt[H + k] = fg; gt[2 * H + k] = gg; gt[3 * H + k] = og;
      hprev[ob + k] = sh[k];
      cst[ob + k] = c;
      out[ob + k] = h;
    }
    __syncthreads();
    for (int k = tid; k < H; k += blockDim.x) {
      sh[k] = out[ob + k];
      sc[k] = cst[ob + k];
    }
    __syncthreads();
  }
  for (int k = tid; k < H; k += blockDim.x) {
    hn[(long)b * H + k] = sh[k];
    cn[(long)b * H + k] = sc[k];
  }
}

// Backward through time.  dout [B][T][H] (may be null = zeros), dhn/dcn [B][H]
// (may be null).  whh [4H][H] (row-major, as stored by nn.LSTM).
// Writes dgates [B][T][4H] (pre-activation gradients).
__global__ __launch_bounds__(256) void lstm_bwd_kernel(const float* __restrict__ dout, const float* __restrict__ dhn,
                                                       const float* __restrict__ dcn, const float* __restrict__ whh,
                                                       const float* __restrict__ cst, const float* __restrict__ gates,
                                                       float* __restrict__ dgates, int T, int H) {
  extern __shared__ float sm[];   // dh [H], dc [H], dgates_t [4H]
  float* sdh = sm;
  float* sdc = sm + H;
  float* sdg = sm + 2 * H;
  const int b = blockIdx.x, tid = threadIdx.x;
  const int G4 = 4 * H;
  for (int k = tid; k < H; k += blockDim.x) {
    sdh[k] = dhn ? dhn[(long)b * H + k] : 0.f;
    sdc[k] = dcn ? dcn[(long)b * H + k] : 0.f;
  }
  __syncthreads();
  for (int t = T - 1; t >= 0; --t) {
    const long ob = ((long)b * T + t) * H;
    const float* gt = gates + ((long)b * T + t) * G4;
    float* dg = dgates + ((long)b * T + t) * G4;
    for (int k = tid; k < H; k += blockDim.x) {
      const float dh = sdh[k] + (dout ? dout[ob + k] : 0.f);
      const float c = cst[ob + k];
      const float cp = t > 0 ? cst[ob - H + k] : 0.f;
      const float ig = gt[k], fg = gt[H + k], gg = gt[2 * H + k], og = gt[3 * H + k];
      const float tc = tanhf(c);
      const float dO = dh * tc;
      const float dc = sdc[k] + dh * og * (1.f - tc * tc);
      const float dI = dc * gg, dG = dc * ig, dF = dc * cp;
      sdc[k] = dc * fg;
      const float a0 = dI * ig * (1.f - ig), a1 = dF * fg * (1.f - fg), a2 = dG * (1.f - gg * gg),
                  a3 = dO * og * (1.f - og);
      sdg[k] = a0; sdg[H + k] = a1; sdg[2 * H + k] = a2; sdg[3 * H + k] = a3;
      dg[k] = a0; dg[H + k] = a1; dg[2 * H + k] = a2; dg[3 * H + k] = a3;
    }
    __syncthreads();
    // dh_{t-1}[k] = sum_j dgates[j] * whh[j][k]
    for (int k = tid; k < H; k += blockDim.x) {
      float acc = 0.f;
      for (int j = 0; j < G4; ++j) acc = fmaf(sdg[j], whh[(long)j * H + k], acc);
      sdh[k] = acc;
    }
    __syncthreads();
  }
}

}  // namespace

extern "C" {

int xcp_lstm_fwd(const float* xproj, const float* whhT, const float* bih, const float* bhh, float* out, float* hprev,
                 float* cst, float* gates, float* hn, float* cn, int B, int T, int H, hipStream_t st) {
  if (B <= 0 || T <= 0) return XCP_OK;
  const size_t smem = (size_t)6 * H * sizeof(float);
  hipLaunchKernelGGL(lstm_fwd_kernel, dim3(B), dim3(256), smem, st, xproj, whhT, bih, bhh, out, hprev, cst, gates, hn, cn,
                     T, H);
  return (int)hipGetLastError();
}

int xcp_lstm_bwd(const float* dout, const float* dhn, const float* dcn, const float* whh, const float* cst,
                 const float* gates, float* dgates, int B, int T, int H, hipStream_t st) {
  if (B <= 0 || T <= 0) return XCP_OK;
  const size_t smem = (size_t)6 * H * sizeof(float);
  hipLaunchKernelGGL(lstm_bwd_kernel, dim3(B), dim3(256), smem, st, dout, dhn, dcn, whh, cst, gates, dgates, T, H);
  return (int)hipGetLastError();
}

}  // extern "C"
