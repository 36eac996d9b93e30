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


// ---------------------------------------------------------------------------------
// Register-resident recurrence for H <= 128 (XceptionLSTMV: H = 128).  One 1024-thread
// workgroup per clip holds the whole W_hh in VGPRs (4H*H/1024 = 64 fp32 per thread at
// H = 128), so a time step is KPT FMAs per thread against h broadcast from LDS, an
// S-lane shuffle reduction and the cell math: no global traffic on the serial path
// except the per-step x-projection / state rows, which are prefetched one step ahead.
//
// forward: thread (gate j, part s), tid = j*S + s, holds W_hh[j][s*KPT .. +KPT).
template <int H>
__global__ __launch_bounds__(1024) void lstm_fwd_reg_kernel(const float* __restrict__ xproj,
                                                            const float* __restrict__ whh,
                                                            const float* __restrict__ bih,
                                                            const float* __restrict__ bhh, float* __restrict__ out,
                                                            float* __restrict__ hprev, float* __restrict__ cst,
                                                            float* __restrict__ gates, float* __restrict__ hn,
                                                            float* __restrict__ cn, int T) {
  constexpr int G4 = 4 * H, S = 1024 / G4, KPT = H / S, PADK = KPT + 4;
  static_assert(S >= 1 && KPT % 4 == 0, "unsupported H");
  __shared__ __attribute__((aligned(16))) float sh[S * PADK];   // h_{t-1}, part s at s*PADK (bank-spread)
  __shared__ float sg[G4];                                      // activated gates of step t
  const int tid = threadIdx.x, b = blockIdx.x;
  const int j = tid / S, s = tid % S;
  float w[KPT];
  const float* wp = whh + (long)j * H + s * KPT;
#pragma unroll
  for (int q = 0; q < KPT; q += 4) {
    const float4 v = *reinterpret_cast<const float4*>(wp + q);
    w[q] = v.x; w[q + 1] = v.y; w[q + 2] = v.z; w[q + 3] = v.w;
  }
  const float bias = bih[j] + bhh[j];
  const bool gate_tanh = (j / H) == 2;
  auto hidx = [](int k) { return (k / KPT) * PADK + k % KPT; };
  if (tid < H) sh[hidx(tid)] = 0.f;
  float c = 0.f;                                 // c_{t-1}[tid] for tid < H
  const float* xb = xproj + (long)b * T * G4;
  float xn = s == 0 ? xb[j] : 0.f;
  __syncthreads();
  for (int t = 0; t < T; ++t) {
    const float xc = xn;
    if (s == 0 && t + 1 < T) xn = xb[(long)(t + 1) * G4 + j];
    float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
    const float* hp = sh + s * PADK;
#pragma unroll
    for (int q = 0; q < KPT; q += 4) {
      const float4 h4 = *reinterpret_cast<const float4*>(hp + q);
      a0 = fmaf(h4.x, w[q], a0);
      a1 = fmaf(h4.y, w[q + 1], a1);
      a2 = fmaf(h4.z, w[q + 2], a2);
      a3 = fmaf(h4.w, w[q + 3], a3);
    }
    float acc = (a0 + a1) + (a2 + a3);
#pragma unroll
    for (int o = 1; o < S; o <<= 1) acc += __shfl_xor(acc, o, 64);
    if (s == 0) {
      const float pre = acc + xc + bias;
      const float v = gate_tanh ? tanhf(pre) : sigm(pre);
      sg[j] = v;
      gates[((long)b * T + t) * G4 + j] = v;
    }
    __syncthreads();
    if (tid < H) {
      const long ob = ((long)b * T + t) * H + tid;
      const float ig = sg[tid], fg = sg[H + tid], gg = sg[2 * H + tid], og = sg[3 * H + tid];
      hprev[ob] = sh[hidx(tid)];
      c = fmaf(fg, c, ig * gg);
      const float h = og * tanhf(c);
      cst[ob] = c;
      out[ob] = h;
      sh[hidx(tid)] = h;      // every read of h_{t-1} happened before the barrier above
    }
    __syncthreads();
  }
  if (tid < H) {
    hn[(long)b * H + tid] = sh[hidx(tid)];
    cn[(long)b * H + tid] = c;
  }
}

// backward: thread (unit k, part p), tid = k*P + p, holds W_hh[p*JPT .. +JPT)[k]; the
// step's pre-activation gradients are broadcast from LDS and dh_{t-1}[k] is reduced over
// the P parts (adjacent lanes) by shuffles.
template <int H>
__global__ __launch_bounds__(1024) void lstm_bwd_reg_kernel(const float* __restrict__ dout,
                                                            const float* __restrict__ dhn,
                                                            const float* __restrict__ dcn,
                                                            const float* __restrict__ whh,
                                                            const float* __restrict__ cst,
                                                            const float* __restrict__ gates,
                                                            float* __restrict__ dgates, int T) {
  constexpr int G4 = 4 * H, P = 1024 / H, JPT = G4 / P, PADJ = JPT + 4;
  static_assert(P >= 1 && JPT % 4 == 0, "unsupported H");
  __shared__ __attribute__((aligned(16))) float sdg[P * PADJ];
  __shared__ float sdh[H];
  const int tid = threadIdx.x, b = blockIdx.x;
  const int k = tid / P, p = tid % P;
  float w[JPT];
#pragma unroll
  for (int q = 0; q < JPT; ++q) w[q] = whh[(long)(p * JPT + q) * H + k];
  auto gidx = [](int jj) { return (jj / JPT) * PADJ + jj % JPT; };
  float dc = 0.f;                                // dc carried into step t, unit tid < H
  // per-step inputs of unit tid, prefetched one step ahead
  float n_c = 0.f, n_cp = 0.f, n_i = 0.f, n_f = 0.f, n_g = 0.f, n_o = 0.f, n_do = 0.f;
  auto fetch = [&](int t) {
    const long ob = ((long)b * T + t) * H + tid;
    const float* gt = gates + ((long)b * T + t) * G4;
    n_c = cst[ob];
    n_cp = t > 0 ? cst[ob - H] : 0.f;
    n_i = gt[tid]; n_f = gt[H + tid]; n_g = gt[2 * H + tid]; n_o = gt[3 * H + tid];
    n_do = dout ? dout[ob] : 0.f;
  };
  if (tid < H) {
    sdh[tid] = dhn ? dhn[(long)b * H + tid] : 0.f;
    dc = dcn ? dcn[(long)b * H + tid] : 0.f;
    fetch(T - 1);
  }
  __syncthreads();
  for (int t = T - 1; t >= 0; --t) {
    if (tid < H) {
      const float c = n_c, cp = n_cp, ig = n_i, fg = n_f, gg = n_g, og = n_o;
      const float dh = sdh[tid] + n_do;
      if (t > 0) fetch(t - 1);
      const float tc = tanhf(c);
      const float dO = dh * tc;
      const float dct = dc + dh * og * (1.f - tc * tc);
      const float dI = dct * gg, dG = dct * ig, dF = dct * cp;
      dc = dct * fg;
      const float g0 = dI * ig * (1.f - ig), g1 = dF * fg * (1.f - fg), g2 = dG * (1.f - gg * gg),
                  g3 = dO * og * (1.f - og);
      float* dg = dgates + ((long)b * T + t) * G4;
      dg[tid] = g0; dg[H + tid] = g1; dg[2 * H + tid] = g2; dg[3 * H + tid] = g3;
      sdg[gidx(tid)] = g0; sdg[gidx(H + tid)] = g1; sdg[gidx(2 * H + tid)] = g2; sdg[gidx(3 * H + tid)] = g3;
    }
    __syncthreads();
    float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
    const float* gp = sdg + p * PADJ;
#pragma unroll
    for (int q = 0; q < JPT; q += 4) {
      const float4 g4 = *reinterpret_cast<const float4*>(gp + q);
      a0 = fmaf(g4.x, w[q], a0);
      a1 = fmaf(g4.y, w[q + 1], a1);
      a2 = fmaf(g4.z, w[q + 2], a2);
      a3 = fmaf(g4.w, w[q + 3], a3);
    }
    float acc = (a0 + a1) + (a2 + a3);
#pragma unroll
    for (int o = 1; o < P; o <<= 1) acc += __shfl_xor(acc, o, 64);
    if (p == 0) sdh[k] = acc;
    __syncthreads();
  }
}

int g_lstm_kernel = 0;   // xcp_tune knob 9: 0 = register-resident kernels where H allows, 1 = generic

bool lstm_reg(int H) { return g_lstm_kernel == 0 && (H == 128 || H == 64); }

}  // namespace

int xcp_internal_lstm_tune(int value) {
  const int old = g_lstm_kernel;
  if (value == 0 || value == 1) g_lstm_kernel = value;
  return old;
}


extern "C" {

// 1 when the recurrence runs on the register-resident kernels (whhT is then unused)
int xcp_lstm_needs_whhT(int H) { return lstm_reg(H) ? 0 : 1; }

int xcp_lstm_fwd(const float* xproj, const float* whh, const float* whhT, const float* bih, const float* bhh, float* out,
                 float* hprev, float* cst, float* gates, float* hn, float* cn, int B, int T, int H, hipStream_t st) {
  if (B <= 0 || T <= 0) return XCP_OK;
  if (lstm_reg(H)) {
    if (H == 128)
      hipLaunchKernelGGL(lstm_fwd_reg_kernel<128>, dim3(B), dim3(1024), 0, st, xproj, whh, bih, bhh, out, hprev, cst,
                         gates, hn, cn, T);
    else
      hipLaunchKernelGGL(lstm_fwd_reg_kernel<64>, dim3(B), dim3(1024), 0, st, xproj, whh, bih, bhh, out, hprev, cst,
                         gates, hn, cn, T);
    return (int)hipGetLastError();
  }
  if (!whhT) return XCP_EINVAL;
  const size_t smem = (size_t)6 * H * sizeof(float);
  hipLaunchKernelGGL(lstm_fwd_kernel, dim3(B), dim3(256), smem, st, xproj, whhT, bih, bhh, out, hprev, cst, gates, hn, cn,
                     T, H);
  return (int)hipGetLastError();
}

int xcp_lstm_bwd(const float* dout, const float* dhn, const float* dcn, const float* whh, const float* cst,
                 const float* gates, float* dgates, int B, int T, int H, hipStream_t st) {
  if (B <= 0 || T <= 0) return XCP_OK;
  if (lstm_reg(H)) {
    if (H == 128)
      hipLaunchKernelGGL(lstm_bwd_reg_kernel<128>, dim3(B), dim3(1024), 0, st, dout, dhn, dcn, whh, cst, gates, dgates,
                         T);
    else
      hipLaunchKernelGGL(lstm_bwd_reg_kernel<64>, dim3(B), dim3(1024), 0, st, dout, dhn, dcn, whh, cst, gates, dgates,
                         T);
    return (int)hipGetLastError();
  }
  const size_t smem = (size_t)6 * H * sizeof(float);
  hipLaunchKernelGGL(lstm_bwd_kernel, dim3(B), dim3(256), smem, st, dout, dhn, dcn, whh, cst, gates, dgates, T, H);
  return (int)hipGetLastError();
}

}  // extern "C"
