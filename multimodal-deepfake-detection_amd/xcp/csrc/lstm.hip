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
#include <stdlib.h>
#include <mutex>
#include <utility>
#include <vector>

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


// ---------------------------------------------------------------------------------
// Per-step kernels for large H (XceptionLSTMA: H = 512, T = 120).  One workgroup per clip
// cannot keep up there: it streams the whole W_hh (4H x H fp32 = 4 MB) through one CU per
// step (~530 us a step).  Here every time step is one launch spread over H / 2 workgroups
// (256 at H = 512), each owning 2 hidden units -- their 8 gate rows of W_hh (forward) or
// their 2 columns (backward); the launch boundary is the grid-wide step barrier and makes
// h_t / dgates_t visible to every CU.
//
// forward step t: thread (row r = gate q of unit uu, k-slice s of H/32) dots its W_hh row
// slice with h_{t-1} (staged in LDS, rows padded against bank conflicts) for every clip,
// the 32 slices reduce by shuffles, and (clip, unit) threads run the cell.
constexpr int LS_UPW = 2;              // hidden units per workgroup
constexpr int LS_MAXB = 32;            // clips (register partials per thread)

template <int KS>   // KS = H / 32 (k values per slice)
__global__ __launch_bounds__(256) void lstm_fwd_step_kernel(const float* __restrict__ xproj, const float* __restrict__ whh,
                                                            const float* __restrict__ bih, const float* __restrict__ bhh,
                                                            float* __restrict__ out, float* __restrict__ hprev,
                                                            float* __restrict__ cst, float* __restrict__ gates,
                                                            float* __restrict__ hn, float* __restrict__ cn, int B, int T,
                                                            int t) {
  constexpr int H = KS * 32, G4 = 4 * H, PS = KS + 4;   // LDS slice pitch (floats)
  constexpr int RP = 33;                                // pitch of a (row, clip) partial row
  extern __shared__ float sm[];   // h_{t-1} [B][32][PS] (then the partials [8][B][RP]), then pre [8][B]
  float* sh = sm;
  float* spre = sm + B * 32 * PS;
  const int tid = threadIdx.x, u0 = blockIdx.x * LS_UPW;
  const int r = tid >> 5, s = tid & 31, q = r >> 1, uu = r & 1;
  const int j = q * H + u0 + uu;
  // W_hh row slice
  float w[KS];
#pragma unroll
  for (int i = 0; i < KS; i += 4) {
    const float4 v = *reinterpret_cast<const float4*>(whh + (long)j * H + s * KS + i);
    w[i] = v.x; w[i + 1] = v.y; w[i + 2] = v.z; w[i + 3] = v.w;
  }
  // stage h_{t-1} (zero at t = 0): 8 loads in flight per thread -- unconditional (clamped index;
  // t = 0 reads step 0's slot as a stand-in and selects zero), since a load under a condition is
  // issued and waited for on its own
  const int n4 = B * H / 4;
  const int tp = t > 0 ? t - 1 : 0;
  for (int e0 = tid; e0 < n4; e0 += 8 * 256) {
    float4 v[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int e = min(e0 + i * 256, n4 - 1);
      const int b = e / (H / 4), k4 = (e - b * (H / 4)) * 4;
      v[i] = *reinterpret_cast<const float4*>(out + ((long)b * T + tp) * H + k4);
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int e = e0 + i * 256;
      const int b = e / (H / 4), k4 = (e - b * (H / 4)) * 4;
      if (e < n4)
        *reinterpret_cast<float4*>(sh + (b * 32 + k4 / KS) * PS + (k4 % KS)) =
            t > 0 ? v[i] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  }
  __syncthreads();
  // every clip's partial dot of this thread's row slice, independent chains (no per-clip
  // cross-lane reduction on the critical path)
  float acc[LS_MAXB];
#pragma unroll
  for (int b = 0; b < LS_MAXB; ++b) {
    acc[b] = 0.f;
    if (b < B) {
      // 16-B reads (ds_read_b128, banks (a/4) % 64): the slices' pitch PS = KS + 4 puts every
      // lane group's 16 slices on distinct 4-bank slots (as 2-dword reads, banks mod 32, the same
      // pitch was a 4-way conflict: 71 % of this kernel's LDS cycles)
      const float4* hb = reinterpret_cast<const float4*>(sh + (b * 32 + s) * PS);
      float a0 = 0.f, a1 = 0.f;
#pragma unroll
      for (int i = 0; i < KS; i += 4) {
        const float4 h4 = hb[i / 4];
        a0 = fmaf(w[i], h4.x, a0);
        a1 = fmaf(w[i + 1], h4.y, a1);
        a0 = fmaf(w[i + 2], h4.z, a0);
        a1 = fmaf(w[i + 3], h4.w, a1);
      }
      acc[b] = a0 + a1;
    }
  }
  __syncthreads();   // h_{t-1} no longer read: its space takes the partials
  float* red = sm;
#pragma unroll
  for (int b = 0; b < LS_MAXB; ++b)
    if (b < B) red[(r * B + b) * RP + s] = acc[b];
  __syncthreads();
  // (row, clip) threads sum the 32 slices in the pairwise order of a 5-level xor butterfly
  if (tid < 8 * B) {
    const float* pr = red + tid * RP;
    float v[32];
#pragma unroll
    for (int i = 0; i < 32; ++i) v[i] = pr[i];
#pragma unroll
    for (int w2 = 1; w2 < 32; w2 <<= 1)
#pragma unroll
      for (int i = 0; i < 32; i += 2 * w2) v[i] = v[i] + v[i + w2];
    spre[tid] = v[0];   // tid = row * B + clip
  }
  __syncthreads();
  if (tid < B * LS_UPW) {
    const int b = tid / LS_UPW, v = tid - b * LS_UPW, k = u0 + v;
    const float* xp = xproj + ((long)b * T + t) * G4;
    float pre[4];
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int jj = g * H + k;
      pre[g] = spre[(g * 2 + v) * B + b] + xp[jj] + bih[jj] + bhh[jj];
    }
    const float ig = sigm(pre[0]), fg = sigm(pre[1]), gg = tanhf(pre[2]), og = sigm(pre[3]);
    const long ob = ((long)b * T + t) * H;
    const long op = t > 0 ? ob - H + k : ob + k;   // t = 0: a valid stand-in, selected away
    const float vcp = cst[op], vhp = out[op];
    const float cp = t > 0 ? vcp : 0.f;
    const float c = fmaf(fg, cp, ig * gg);
    const float h = og * tanhf(c);
    float* gt = gates + ((long)b * T + t) * G4;
    gt[k] = ig; gt[H + k] = fg; gt[2 * H + k] = gg; gt[3 * H + k] = og;
    hprev[ob + k] = t > 0 ? vhp : 0.f;
    cst[ob + k] = c;
    out[ob + k] = h;
    if (t == T - 1) {
      hn[(long)b * H + k] = h;
      cn[(long)b * H + k] = c;
    }
  }
}

// whhT[k][j] = whh[j][k] (once per backward call, so a workgroup's W_hh columns are rows)
__global__ __launch_bounds__(256) void lstm_transpose_kernel(const float* __restrict__ whh, float* __restrict__ whhT,
                                                             int H) {
  __shared__ float tl[32][33];
  const int G4 = 4 * H;
  const int j0 = blockIdx.x * 32, k0 = blockIdx.y * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  for (int r = ty; r < 32; r += 8) tl[r][tx] = whh[(long)(j0 + r) * H + k0 + tx];
  __syncthreads();
  for (int r = ty; r < 32; r += 8) whhT[(long)(k0 + r) * G4 + j0 + tx] = tl[tx][r];
}

// backward step t: dh_t[b][k] = dout[b][t][k] + sum_j dgates_{t+1}[b][j] W_hh[j][k] (dhn at
// t = T-1): thread (clip b, j-slice sl of 4H/16) against the workgroup's 2 W_hh columns in
// LDS, 16-slice shuffle reduction; (clip, unit) threads run the cell backward with the cell
// gradient carried in dcw [B][H] (each unit's carry is only touched by its workgroup).
__global__ __launch_bounds__(256) void lstm_bwd_step_kernel(const float* __restrict__ dout, const float* __restrict__ dhn,
                                                            const float* __restrict__ dcn, const float* __restrict__ whhT,
                                                            const float* __restrict__ cst, const float* __restrict__ gates,
                                                            float* __restrict__ dgates, float* __restrict__ dcw, int B,
                                                            int T, int H, int t) {
  extern __shared__ float sm[];   // W columns [16 slices][SP] ([4H / 16][2] each), dh [B][2]
  const int G4 = 4 * H;
  const int per = G4 / 16, SP = 2 * per + 4;   // slice pitch: +4 floats, so the 16 slices of a
                                               // half-wave start on 16 different 4-bank groups
  float* swc = sm;
  float* sdh = sm + 16 * SP;
  const int tid = threadIdx.x, u0 = blockIdx.x * LS_UPW;
  if (t < T - 1) {
    // rows u0, u0+1 of W_hh^T (contiguous), interleaved into swc[j][2]: 16-B loads, up to 4 per
    // row per thread issued before any store (clamped indices; a loop of dependent scalar loads
    // was ~8 L2 round trips a step at H = 512)
    const int n4 = G4 / 4;
    const float4* r0 = reinterpret_cast<const float4*>(whhT + (long)u0 * G4);
    const float4* r1 = reinterpret_cast<const float4*>(whhT + (long)(u0 + 1) * G4);
    for (int e0 = tid; e0 < n4; e0 += 4 * 256) {
      float4 x0[4], x1[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int e = min(e0 + i * 256, n4 - 1);
        x0[i] = r0[e];
        x1[i] = r1[e];
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int e = e0 + i * 256;
        if (e < n4) {   // jj = 4e..4e+3, all in slice 4e / per
          float4* d = reinterpret_cast<float4*>(swc + (4 * e / per) * SP + 2 * (4 * e % per));
          d[0] = make_float4(x0[i].x, x1[i].x, x0[i].y, x1[i].y);
          d[1] = make_float4(x0[i].z, x1[i].z, x0[i].w, x1[i].w);
        }
      }
    }
    __syncthreads();
    for (int b0 = 0; b0 < B; b0 += 16) {
      const int b = b0 + (tid >> 4), sl = tid & 15;
      float a0 = 0.f, a1 = 0.f;
      if (b < B) {
        const float* dg = dgates + ((long)b * T + t + 1) * G4 + sl * per;
        const float* wc = swc + sl * SP;
        // 16 independent 16-B loads in flight per batch (the loop is L2-latency-bound otherwise)
        for (int i0 = 0; i0 < per; i0 += 64) {
          float4 g4[16];
#pragma unroll
          for (int q = 0; q < 16; ++q) g4[q] = *reinterpret_cast<const float4*>(dg + i0 + 4 * q);
#pragma unroll
          for (int q = 0; q < 16; ++q) {
            const float gv[4] = {g4[q].x, g4[q].y, g4[q].z, g4[q].w};
            // (W[i][0], W[i][1], W[i+1][0], W[i+1][1]) as one ds_read_b128: banks (a/4) % 64, the
            // 16 slices 4 banks apart (pitch SP), so a lane group's reads never collide
            const float4* w4 = reinterpret_cast<const float4*>(wc + 2 * (i0 + 4 * q));
            const float4 wa = w4[0], wb = w4[1];
            const float wv[8] = {wa.x, wa.y, wa.z, wa.w, wb.x, wb.y, wb.z, wb.w};
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              a0 = fmaf(gv[e], wv[2 * e], a0);
              a1 = fmaf(gv[e], wv[2 * e + 1], a1);
            }
          }
        }
      }
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) {
        a0 += __shfl_xor(a0, o, 64);
        a1 += __shfl_xor(a1, o, 64);
      }
      if (sl == 0 && b < B) {
        sdh[b * 2] = a0;
        sdh[b * 2 + 1] = a1;
      }
    }
    __syncthreads();
  }
  if (tid < B * LS_UPW) {
    const int b = tid / LS_UPW, v = tid - b * LS_UPW, k = u0 + v;
    const long ob = ((long)b * T + t) * H, bk = (long)b * H + k;
    // every global load unconditional (absent operands read a valid stand-in address and are
    // selected away), so they go out together instead of one round trip per branch
    const bool last = t == T - 1;
    const float* pc = cst + ob + k;
    const float vhn = *(last && dhn ? dhn + bk : pc);
    const float vcw = *(!last ? dcw + bk : (dcn ? dcn + bk : pc));
    const float vdo = *(dout ? dout + ob + k : pc);
    const float vcp = *(t > 0 ? pc - H : pc);
    const float c = *pc;
    const float* gt = gates + ((long)b * T + t) * G4;
    const float ig = gt[k], fg = gt[H + k], gg = gt[2 * H + k], og = gt[3 * H + k];
    const float dhr = !last ? sdh[b * 2 + v] : (dhn ? vhn : 0.f);
    const float dcr = !last || dcn ? vcw : 0.f;
    const float dh = dhr + (dout ? vdo : 0.f);
    const float cp = t > 0 ? vcp : 0.f;
    const float tc = tanhf(c);
    const float dO = dh * tc;
    const float dc = dcr + dh * og * (1.f - tc * tc);
    const float dI = dc * gg, dG = dc * ig, dF = dc * cp;
    dcw[bk] = dc * fg;
    float* dg = dgates + ((long)b * T + t) * G4;
    dg[k] = dI * ig * (1.f - ig);
    dg[H + k] = dF * fg * (1.f - fg);
    dg[2 * H + k] = dG * (1.f - gg * gg);
    dg[3 * H + k] = dO * og * (1.f - og);
  }
}

// ---------------------------------------------------------------------------------
// Persistent recurrence for H = 256 / 512 (XceptionLSTMA: H = 512, T = 120): ONE launch per
// direction walks all T steps, instead of the T launches of the per-step kernels above (each of
// which re-read its W_hh slice from L2 and paid a kernel boundary per step).
//
// G = H / 4 workgroups of 256 threads, each owning 4 hidden units for the whole launch, with
// their W_hh slice in VGPRs (one wave per SIMD, 128 fp32 weights per lane):
//   forward : lane l holds W_hh[16 gate rows of its units][k = l*KL .. +KL)  (KL = H / 64)
//   backward: lane l holds W_hh[j = l*JL .. +JL)[its 4 units]              (JL = 4H / 64)
// Wave v handles clips 16p + 4v .. +3 (pass p = 0, 1 for B <= 32).  A step's dot products are
// per-lane FMA chains over the lane's k (j) range; the 64 lanes' partial sums (16 rows x 4 clips
// forward, 4 units x 4 clips backward) are combined by a reduce-scatter butterfly (each xor level
// halves what a lane keeps), so after 6 levels lane l holds one complete (clip, row) sum
// (forward: clip l >> 4, row l & 15 = gate * 4 + unit; backward: clip l >> 4, unit (l >> 2) & 3).
// The cell runs on 16 lanes per wave with c (forward) / the cell-gradient carry (backward) kept
// in a register across steps.
// Step hand-off (guide: MI355X_MICROARCH.md "Valid forms", first table row): every store of
// h_t (forward) / dgates_t (backward) is a 4-B sc1 store; each storing wave waits vmcnt(0),
// the workgroup barriers, and one lane adds 1 to its shard counter (blockIdx % 8, one 128-B line
// each, agent-scope atomic).  Before a step, wave 0 polls the 8 shards with sc1 loads until each
// counted every one of its workgroups for the previous step, the workgroup barriers, and every
// load of the handed-off values is a 16-B sc1 buffer load.  Counters are zeroed by the host per
// launch; a poll that runs past ~LP_SPIN sleeps sets the error word and the workgroup leaves
// (the results are then invalid, but no wave spins forever: e.g. if fewer than G workgroups
// could ever be resident, which the host rules out with the occupancy query).
constexpr int LP_U = 4;                   // hidden units per workgroup
constexpr int LP_SHARD = 32;              // uints per shard counter (one 128-B line)
constexpr unsigned LP_SPIN = 1u << 22;    // polls (each after s_sleep 2) before giving up
constexpr int LP_CSP = 0x00020000;        // raw buffer descriptor word 3
constexpr int LP_SC1 = 16;                // cache policy: sc1

typedef int i32x4v __attribute__((ext_vector_type(4)));

struct LstmSync {
  unsigned* cnt;   // [8][LP_SHARD]
  unsigned* err;   // set to 1 on a poll timeout
};

// wave 0 waits until every shard has `steps` arrivals from each of its workgroups; then the
// workgroup barrier.  false (every thread) on a timeout.
XCP_DEV bool lp_wait(const LstmSync& sy, unsigned steps) {
  __shared__ int s_ok;
  const int tid = threadIdx.x, lane = tid & 63, G = gridDim.x;
  if (tid < 64) {
    const unsigned want = steps * (unsigned)(G / 8 + ((lane & 7) < G % 8 ? 1 : 0));
    unsigned it = 0;
    bool ok = false;
    while (true) {
      const unsigned v = lane < 8 ? __hip_atomic_load(sy.cnt + lane * LP_SHARD, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                  : want;
      ok = __all(v >= want);
      if (ok || ++it > LP_SPIN) break;
      __builtin_amdgcn_s_sleep(2);
    }
    if (tid == 0) {
      s_ok = ok;
      if (!ok) __hip_atomic_store(sy.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  __syncthreads();
  return s_ok != 0;
}

// every wave's sc1 stores have completed; then one arrival on this workgroup's shard
XCP_DEV void lp_publish(const LstmSync& sy) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0)
    __hip_atomic_fetch_add(sy.cnt + (blockIdx.x % 8) * LP_SHARD, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

XCP_DEV void lp_st(float* p, float v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }

template <int V> struct LpIC {
  static constexpr int value = V;
};
template <int B, int E, typename F>
XCP_DEV void lp_static_for(F&& f) {
  if constexpr (B < E) {
    f(LpIC<B>{});
    lp_static_for<B + 1, E>(f);
  }
}

// reduce-scatter of v[N] over the 64 lanes: level d keeps the upper half where lane & d; after
// log2(N) levels lane l holds index (l >> (6 - log2 N)) complete over those lanes, the remaining
// levels sum plainly (every lane of a group ends with the same value).  Every index is a
// compile-time constant (the array stays in VGPRs).
template <int N>
XCP_DEV float lp_rscatter(float (&v)[N], int lane) {
  lp_static_for<0, 6>([&](auto L) {
    constexpr int d = 32 >> decltype(L)::value;
    constexpr int n = N >> decltype(L)::value;
    if constexpr (n >= 2) {
      const bool up = lane & d;
#pragma unroll
      for (int c = 0; c < n / 2; ++c) {
        const float keep = up ? v[n / 2 + c] : v[c];
        const float send = up ? v[c] : v[n / 2 + c];
        v[c] = keep + __shfl_xor(send, d, 64);
      }
    } else {
      v[0] += __shfl_xor(v[0], d, 64);
    }
  });
  return v[0];
}

// (one wave per SIMD: the whole 512-entry register file, so a step's loads all go out before the
// first use -- at 256 registers hipcc issued them clip by clip, one L2 round trip each)
template <int H>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1)))
void lstm_fwd_persist_kernel(const float* __restrict__ xproj, const float* __restrict__ whh,
                             const float* __restrict__ bih, const float* __restrict__ bhh, float* out,
                             float* __restrict__ hprev, float* __restrict__ cst, float* __restrict__ gates,
                             float* __restrict__ hn, float* __restrict__ cn, int B, int T, LstmSync sy) {
  constexpr int KL = H / 64, R = 4 * LP_U, G4 = 4 * H;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int u0 = blockIdx.x * LP_U, k0 = lane * KL;
  float w[R][KL];
#pragma unroll
  for (int rr = 0; rr < R; ++rr)
#pragma unroll
    for (int i = 0; i < KL; i += 4) {
      const float4 v4 = *reinterpret_cast<const float4*>(whh + (long)((rr / LP_U) * H + u0 + rr % LP_U) * H + k0 + i);
      w[rr][i] = v4.x; w[rr][i + 1] = v4.y; w[rr][i + 2] = v4.z; w[rr][i + 3] = v4.w;
    }
  // cell lanes: lane = c * 16 + u (gate 0 of unit u of clip c); the other gates at lane + 4q
  const bool cell = (lane & 12) == 0;
  const int cu = lane & 3, k = u0 + cu;
  float bi[4], bh[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    bi[q] = bih[q * H + k];
    bh[q] = bhh[q * H + k];
  }
  const int npass = (B + 15) / 16;
  float cstate[2] = {0.f, 0.f}, hst[2] = {0.f, 0.f}, xq[2][4];
  const __amdgpu_buffer_rsrc_t rO = __builtin_amdgcn_make_buffer_rsrc(out, (short)0, 0x7fffffff, LP_CSP);
  auto clip = [&](int p, int c) { return p * 16 + wv * 4 + c; };
  auto load_xp = [&](int t) {   // x W_ih^T of step t for this lane's cell (prefetched a step ahead; clamped)
    const int tt = min(t, T - 1);
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      const int b = min(clip(p, lane >> 4), B - 1);
#pragma unroll
      for (int q = 0; q < 4; ++q) xq[p][q] = xproj[((long)b * T + tt) * G4 + q * H + k];
    }
  };
  load_xp(0);
  for (int t = 0; t < T; ++t) {
    float xc[2][4];
#pragma unroll
    for (int p = 0; p < 2; ++p)
#pragma unroll
      for (int q = 0; q < 4; ++q) xc[p][q] = xq[p][q];
    load_xp(t + 1);
    if (t > 0 && !lp_wait(sy, (unsigned)t)) return;
    for (int p = 0; p < npass; ++p) {
      float hv[4][KL];
      if (t > 0) {   // h_{t-1} of the wave's 4 clips (clamped), every 16-B sc1 load issued before any use
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const int b = min(clip(p, c), B - 1);
#pragma unroll
          for (int i = 0; i < KL; i += 4) {
            const float4 v4 = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(
                rO, (int)((((long)b * T + t - 1) * H + k0 + i) * 4), 0, LP_SC1));
            hv[c][i] = v4.x; hv[c][i + 1] = v4.y; hv[c][i + 2] = v4.z; hv[c][i + 3] = v4.w;
          }
        }
      } else {
#pragma unroll
        for (int c = 0; c < 4; ++c)
#pragma unroll
          for (int i = 0; i < KL; ++i) hv[c][i] = 0.f;
      }
      float part[4 * R];
#pragma unroll
      for (int c = 0; c < 4; ++c)
#pragma unroll
        for (int rr = 0; rr < R; ++rr) {
          float a0 = 0.f, a1 = 0.f;
#pragma unroll
          for (int i = 0; i < KL; i += 2) {
            a0 = fmaf(w[rr][i], hv[c][i], a0);
            a1 = fmaf(w[rr][i + 1], hv[c][i + 1], a1);
          }
          part[c * R + rr] = a0 + a1;
        }
      const float rec = lp_rscatter(part, lane);   // clip lane >> 4, row lane & 15
      float pre[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) pre[q] = __shfl(rec, (lane & ~15) | (q * 4 + cu), 64);
      const int b = clip(p, lane >> 4);
      if (cell && b < B) {
        float g[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) g[q] = ((pre[q] + xc[p][q]) + bi[q]) + bh[q];
        const float ig = sigm(g[0]), fg = sigm(g[1]), gg = tanhf(g[2]), og = sigm(g[3]);
        const float c = fmaf(fg, cstate[p], ig * gg);
        const float h = og * tanhf(c);
        const long ob = ((long)b * T + t) * H;
        float* gt = gates + ((long)b * T + t) * G4;
        gt[k] = ig; gt[H + k] = fg; gt[2 * H + k] = gg; gt[3 * H + k] = og;
        hprev[ob + k] = hst[p];
        cst[ob + k] = c;
        lp_st(out + ob + k, h);
        if (t == T - 1) {
          hn[(long)b * H + k] = h;
          cn[(long)b * H + k] = c;
        }
        cstate[p] = c;
        hst[p] = h;
      }
    }
    if (t + 1 < T) lp_publish(sy);
  }
}

// Backward: dh_t[b][k] = dout + sum_j dgates_{t+1}[b][j] W_hh[j][k] needs every gate row j, so instead of
// gathering dgates_{t+1} (B x 4H floats) into every workgroup, each workgroup turns ITS 16 rows'
// dgates into a partial of dh for all H units -- lane l: part[b][k = l*KL .. +KL) = sum over its rows
// of dgates[b][row] W_hh[row][k] (the forward's W slice, the row values broadcast from the cell lanes
// by readlane) -- and publishes it (4 KB per clip, sc1); the next step gathers its 4 units' columns
// of the G partials (16 B per clip and producer) and reduces them over the wave.  Per step and
// workgroup: B x H x 4 B out and B x 16 x G B in (at B = 16, 32 KB each way) instead of B x 4H x 4 B in.
// part: [2 (step parity)][B][H / 4 (unit group)][G (producer)][4] fp32 (the caller's work buffer): a reader's
// gather (its unit group, every producer) is one contiguous 16 x G-byte run per clip, the writes are 16-B
// pieces G x 16 B apart (fire-and-forget; only the publish waits for them).
template <int H>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1)))
void lstm_bwd_persist_kernel(const float* __restrict__ dout, const float* __restrict__ dhn,
                             const float* __restrict__ dcn, const float* __restrict__ whh,
                             const float* __restrict__ cst, const float* __restrict__ gates,
                             float* __restrict__ dgates, float* part, int B, int T, LstmSync sy) {
  constexpr int KL = H / 64, R = 4 * LP_U, G4 = 4 * H;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, G = gridDim.x;
  const int u0 = blockIdx.x * LP_U, k0 = lane * KL;
  float w[R][KL];   // W_hh[gate q, unit u0 + u][k0 .. k0+KL), row rr = q * 4 + u
#pragma unroll
  for (int rr = 0; rr < R; ++rr)
#pragma unroll
    for (int i = 0; i < KL; i += 4) {
      const float4 v4 = *reinterpret_cast<const float4*>(whh + (long)((rr / LP_U) * H + u0 + rr % LP_U) * H + k0 + i);
      w[rr][i] = v4.x; w[rr][i + 1] = v4.y; w[rr][i + 2] = v4.z; w[rr][i + 3] = v4.w;
    }
  // cell lanes: lane = c * 16 + u * 4 (clip c of the wave, unit u)
  const bool cell = (lane & 3) == 0;
  const int cu = (lane >> 2) & 3, k = u0 + cu;
  const int npass = (B + 15) / 16;
  const long pstride = (long)G * B * H;   // one parity's partials
  float carry[2] = {0.f, 0.f};
  const __amdgpu_buffer_rsrc_t rP = __builtin_amdgcn_make_buffer_rsrc(part, (short)0, 0x7fffffff, LP_CSP);
  auto clip = [&](int p, int c) { return p * 16 + wv * 4 + c; };
  for (int t = T - 1; t >= 0; --t) {
    const bool last = t == T - 1;
    // this step's cell operands (independent of the recurrence: loaded before the wait; clamped
    // addresses, absent operands selected away)
    float vc[2], vcp[2], vg[2][4], vdo[2], vhn[2], vcn[2];
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      const int b = min(clip(p, lane >> 4), B - 1);
      const long ob = ((long)b * T + t) * H + k, bk = (long)b * H + k;
      vc[p] = cst[ob];
      vcp[p] = cst[t > 0 ? ob - H : ob];
      vdo[p] = *(dout ? dout + ob : cst + ob);
      vhn[p] = *(dhn ? dhn + bk : cst + ob);
      vcn[p] = *(dcn ? dcn + bk : cst + ob);
#pragma unroll
      for (int q = 0; q < 4; ++q) vg[p][q] = gates[((long)b * T + t) * G4 + q * H + k];
      if (t == 0) vcp[p] = 0.f;
      if (!dout) vdo[p] = 0.f;
      if (!dhn) vhn[p] = 0.f;
      if (!dcn) vcn[p] = 0.f;
    }
    if (!last && !lp_wait(sy, (unsigned)(T - 1 - t))) return;
    for (int p = 0; p < npass; ++p) {
      if (clip(p, 0) >= B) continue;   // (wave-uniform: no clip of this wave in this pass)
      float red[4 * LP_U];
      if (!last) {   // this workgroup's 4 units of the G partials of step t+1: lanes l and l + 64
        const float* pp = part + (long)((t + 1) & 1) * pstride;
        float4 pv[4][2];
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const int b = min(clip(p, c), B - 1);
#pragma unroll
          for (int e = 0; e < 2; ++e) {
            const int src = min(lane + 64 * e, G - 1);
            pv[c][e] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(
                rP, (int)((((long)((t + 1) & 1) * pstride + (((long)b * (H / 4) + blockIdx.x) * G + src) * 4) * 4)), 0,
                LP_SC1));
          }
        }
        (void)pp;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const bool e1 = lane + 64 < G;
          red[c * 4 + 0] = pv[c][0].x + (e1 ? pv[c][1].x : 0.f);
          red[c * 4 + 1] = pv[c][0].y + (e1 ? pv[c][1].y : 0.f);
          red[c * 4 + 2] = pv[c][0].z + (e1 ? pv[c][1].z : 0.f);
          red[c * 4 + 3] = pv[c][0].w + (e1 ? pv[c][1].w : 0.f);
          if (lane >= G) red[c * 4] = red[c * 4 + 1] = red[c * 4 + 2] = red[c * 4 + 3] = 0.f;
        }
      } else {
#pragma unroll
        for (int q = 0; q < 4 * LP_U; ++q) red[q] = 0.f;
      }
      const float rec = lp_rscatter(red, lane);   // clip lane >> 4, unit (lane >> 2) & 3
      const int b = clip(p, lane >> 4);
      float dg[4] = {0.f, 0.f, 0.f, 0.f};
      if (cell && b < B) {
        const float ig = vg[p][0], fg = vg[p][1], gg = vg[p][2], og = vg[p][3];
        const float dhr = !last ? rec : vhn[p];
        const float dcr = !last ? carry[p] : vcn[p];
        const float dh = dhr + vdo[p];
        const float tc = tanhf(vc[p]);
        const float dO = dh * tc;
        const float dc = dcr + dh * og * (1.f - tc * tc);
        const float dI = dc * gg, dG = dc * ig, dF = dc * vcp[p];
        carry[p] = dc * fg;
        dg[0] = dI * ig * (1.f - ig);
        dg[1] = dF * fg * (1.f - fg);
        dg[2] = dG * (1.f - gg * gg);
        dg[3] = dO * og * (1.f - og);
        float* dgo = dgates + ((long)b * T + t) * G4;
#pragma unroll
        for (int q = 0; q < 4; ++q) dgo[q * H + k] = dg[q];
      }
      if (t > 0) {   // this workgroup's partial of dh_{t-1} for the wave's clips, every unit k0 .. k0+KL
        float* pw = part + (long)(t & 1) * pstride + (long)blockIdx.x * B * H;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const int bc = clip(p, c);
          float acc[KL];
#pragma unroll
          for (int i = 0; i < KL; ++i) acc[i] = 0.f;
#pragma unroll
          for (int rr = 0; rr < R; ++rr) {   // dgates[bc][gate q, unit u] from cell lane c * 16 + u * 4
            const float d = __builtin_bit_cast(float, __builtin_amdgcn_readlane(
                __builtin_bit_cast(int, dg[rr / LP_U]), c * 16 + (rr % LP_U) * 4));
#pragma unroll
            for (int i = 0; i < KL; ++i) acc[i] = fmaf(d, w[rr][i], acc[i]);
          }
          if (bc < B) {   // units k0 + i .. +3 = unit group (k0 + i) / 4 of this producer
#pragma unroll
            for (int i = 0; i < KL; i += 4)
              __builtin_amdgcn_raw_buffer_store_b128(
                  __builtin_bit_cast(i32x4v, make_float4(acc[i], acc[i + 1], acc[i + 2], acc[i + 3])), rP,
                  (int)(((long)(t & 1) * pstride + (((long)bc * (H / 4) + (k0 + i) / 4) * G + blockIdx.x) * 4) * 4), 0,
                  LP_SC1);
          }
          (void)pw;
        }
      }
    }
    if (t > 0) lp_publish(sy);
  }
}

// Backward, gather form (XCP_LSTM_BWD=gather): each workgroup keeps its 4 units' COLUMNS of W_hh (lane l:
// rows j = l*JL .. +JL, JL = 4H / 64) and gathers the whole dgates_{t+1} of its wave's 4 clips each step
// (every 16-B sc1 load of the step issued before the first use: 512-register waves); per-lane FMA chains,
// reduce-scatter over the wave; it publishes only its own dgates_t (16 floats per clip).
template <int H>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1)))
void lstm_bwd_gather_kernel(const float* __restrict__ dout, const float* __restrict__ dhn,
                            const float* __restrict__ dcn, const float* __restrict__ whh,
                            const float* __restrict__ cst, const float* __restrict__ gates, float* dgates, int B,
                            int T, LstmSync sy) {
  constexpr int JL = 4 * H / 64, G4 = 4 * H;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int u0 = blockIdx.x * LP_U, j0 = lane * JL;
  float w[JL][LP_U];
#pragma unroll
  for (int i = 0; i < JL; ++i) {
    const float4 v4 = *reinterpret_cast<const float4*>(whh + (long)(j0 + i) * H + u0);
    w[i][0] = v4.x; w[i][1] = v4.y; w[i][2] = v4.z; w[i][3] = v4.w;
  }
  const bool cell = (lane & 3) == 0;   // lane = c * 16 + u * 4 (clip c, unit u)
  const int cu = (lane >> 2) & 3, k = u0 + cu;
  const int npass = (B + 15) / 16;
  float carry[2] = {0.f, 0.f};
  const __amdgpu_buffer_rsrc_t rG = __builtin_amdgcn_make_buffer_rsrc(dgates, (short)0, 0x7fffffff, LP_CSP);
  auto clip = [&](int p, int c) { return p * 16 + wv * 4 + c; };
  for (int t = T - 1; t >= 0; --t) {
    const bool last = t == T - 1;
    float vc[2], vcp[2], vg[2][4], vdo[2], vhn[2], vcn[2];
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      const int b = min(clip(p, lane >> 4), B - 1);
      const long ob = ((long)b * T + t) * H + k, bk = (long)b * H + k;
      vc[p] = cst[ob];
      vcp[p] = cst[t > 0 ? ob - H : ob];
      vdo[p] = *(dout ? dout + ob : cst + ob);
      vhn[p] = *(dhn ? dhn + bk : cst + ob);
      vcn[p] = *(dcn ? dcn + bk : cst + ob);
#pragma unroll
      for (int q = 0; q < 4; ++q) vg[p][q] = gates[((long)b * T + t) * G4 + q * H + k];
      if (t == 0) vcp[p] = 0.f;
      if (!dout) vdo[p] = 0.f;
      if (!dhn) vhn[p] = 0.f;
      if (!dcn) vcn[p] = 0.f;
    }
    if (!last && !lp_wait(sy, (unsigned)(T - 1 - t))) return;
    for (int p = 0; p < npass; ++p) {
      if (clip(p, 0) >= B) continue;   // (wave-uniform)
      float part[4 * LP_U];
      if (!last) {
        float dg[4][JL];
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const int b = min(clip(p, c), B - 1);
#pragma unroll
          for (int i = 0; i < JL; i += 4) {
            const float4 v4 = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(
                rG, (int)((((long)b * T + t + 1) * G4 + j0 + i) * 4), 0, LP_SC1));
            dg[c][i] = v4.x; dg[c][i + 1] = v4.y; dg[c][i + 2] = v4.z; dg[c][i + 3] = v4.w;
          }
        }
#pragma unroll
        for (int c = 0; c < 4; ++c)
#pragma unroll
          for (int u = 0; u < LP_U; ++u) {
            float a0 = 0.f, a1 = 0.f;
#pragma unroll
            for (int i = 0; i < JL; i += 2) {
              a0 = fmaf(dg[c][i], w[i][u], a0);
              a1 = fmaf(dg[c][i + 1], w[i + 1][u], a1);
            }
            part[c * LP_U + u] = a0 + a1;
          }
      } else {
#pragma unroll
        for (int q = 0; q < 4 * LP_U; ++q) part[q] = 0.f;
      }
      const float rec = lp_rscatter(part, lane);   // clip lane >> 4, unit (lane >> 2) & 3
      const int b = clip(p, lane >> 4);
      if (cell && b < B) {
        const float ig = vg[p][0], fg = vg[p][1], gg = vg[p][2], og = vg[p][3];
        const float dhr = !last ? rec : vhn[p];
        const float dcr = !last ? carry[p] : vcn[p];
        const float dh = dhr + vdo[p];
        const float tc = tanhf(vc[p]);
        const float dO = dh * tc;
        const float dc = dcr + dh * og * (1.f - tc * tc);
        const float dI = dc * gg, dG = dc * ig, dF = dc * vcp[p];
        carry[p] = dc * fg;
        float* dgo = dgates + ((long)b * T + t) * G4;
        lp_st(dgo + k, dI * ig * (1.f - ig));
        lp_st(dgo + H + k, dF * fg * (1.f - fg));
        lp_st(dgo + 2 * H + k, dG * (1.f - gg * gg));
        lp_st(dgo + 3 * H + k, dO * og * (1.f - og));
      }
    }
    if (t > 0) lp_publish(sy);
  }
}

// Backward, clip-grouped gather form (XCP_LSTM_BWD=cg / cg2): the gather kernel's workgroups split by clips as
// well -- workgroup (unit group ug, clip group cg) keeps its 4 units' columns of W_hh and each of its 4
// waves gathers CPW clips' dgates_{t+1} (8 CPW 16-B sc1 loads per lane instead of 32), at H / 4 x
// ceil(B / (4 CPW)) workgroups (CPW 1: two per CU at B = 16, H = 512 -- 128-VGPR weights + one clip's 32
// dgates per lane fit the 256 registers of two waves per SIMD; CPW 2: one per CU).  CPW = 4 with one clip
// group is the gather kernel.
// Per-lane partial chains, reduce-scatter tree and cell update are the gather kernel's, so dgates are
// bitwise its.
template <int H, int CPW>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(CPW == 1 ? 2 : 1, CPW == 1 ? 2 : 1)))
void lstm_bwd_cg_kernel(const float* __restrict__ dout, const float* __restrict__ dhn,
                        const float* __restrict__ dcn, const float* __restrict__ whh,
                        const float* __restrict__ cst, const float* __restrict__ gates, float* dgates, int B,
                        int T, LstmSync sy) {
  constexpr int JL = 4 * H / 64, G4 = 4 * H, NG = H / LP_U, NP = CPW * LP_U;
  constexpr int SH = CPW == 1 ? 4 : CPW == 2 ? 3 : 2;   // lane >> SH: index c * LP_U + u after the reduce-scatter
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int ug = blockIdx.x % NG, cgp = blockIdx.x / NG;
  const int u0 = ug * LP_U, j0 = lane * JL;
  float w[JL][LP_U];
#pragma unroll
  for (int i = 0; i < JL; ++i) {
    const float4 v4 = *reinterpret_cast<const float4*>(whh + (long)(j0 + i) * H + u0);
    w[i][0] = v4.x; w[i][1] = v4.y; w[i][2] = v4.z; w[i][3] = v4.w;
  }
  // this wave's clips (cgp * 4 + wv) * CPW + c; clips past B idle, but keep every barrier
  const int cb = (cgp * 4 + wv) * CPW;
  const int idx = lane >> SH;
  const bool cell = (lane & ((1 << SH) - 1)) == 0;   // lane = (c * LP_U + u) << SH
  const int b = cb + idx / LP_U, k = u0 + idx % LP_U;
  const bool bok = b < B;
  const int bb = bok ? b : B - 1;
  float carry = 0.f;
  const __amdgpu_buffer_rsrc_t rG = __builtin_amdgcn_make_buffer_rsrc(dgates, (short)0, 0x7fffffff, LP_CSP);
  for (int t = T - 1; t >= 0; --t) {
    const bool last = t == T - 1;
    const long ob = ((long)bb * T + t) * H + k, bk = (long)bb * H + k;
    const float vc = cst[ob];
    float vcp = cst[t > 0 ? ob - H : ob];
    float vdo = *(dout ? dout + ob : cst + ob);
    float vhn = *(dhn ? dhn + bk : cst + ob);
    float vcn = *(dcn ? dcn + bk : cst + ob);
    float vg[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) vg[q] = gates[((long)bb * T + t) * G4 + q * H + k];
    if (t == 0) vcp = 0.f;
    if (!dout) vdo = 0.f;
    if (!dhn) vhn = 0.f;
    if (!dcn) vcn = 0.f;
    if (!last && !lp_wait(sy, (unsigned)(T - 1 - t))) return;
    float part[NP];
    if (!last) {
      float dg[CPW][JL];
#pragma unroll
      for (int c = 0; c < CPW; ++c) {
        const int bc = min(cb + c, B - 1);
#pragma unroll
        for (int i = 0; i < JL; i += 4) {
          const float4 v4 = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(
              rG, (int)((((long)bc * T + t + 1) * G4 + j0 + i) * 4), 0, LP_SC1));
          dg[c][i] = v4.x; dg[c][i + 1] = v4.y; dg[c][i + 2] = v4.z; dg[c][i + 3] = v4.w;
        }
      }
#pragma unroll
      for (int c = 0; c < CPW; ++c)
#pragma unroll
        for (int u = 0; u < LP_U; ++u) {
          float a0 = 0.f, a1 = 0.f;
#pragma unroll
          for (int i = 0; i < JL; i += 2) {
            a0 = fmaf(dg[c][i], w[i][u], a0);
            a1 = fmaf(dg[c][i + 1], w[i + 1][u], a1);
          }
          part[c * LP_U + u] = a0 + a1;
        }
    } else {
#pragma unroll
      for (int q = 0; q < NP; ++q) part[q] = 0.f;
    }
    const float rec = lp_rscatter(part, lane);   // index lane >> SH
    if (cell && bok) {
      const float ig = vg[0], fg = vg[1], gg = vg[2], og = vg[3];
      const float dhr = !last ? rec : vhn;
      const float dcr = !last ? carry : vcn;
      const float dh = dhr + vdo;
      const float tc = tanhf(vc);
      const float dO = dh * tc;
      const float dc = dcr + dh * og * (1.f - tc * tc);
      const float dI = dc * gg, dG = dc * ig, dF = dc * vcp;
      carry = dc * fg;
      float* dgo = dgates + ((long)b * T + t) * G4;
      lp_st(dgo + k, dI * ig * (1.f - ig));
      lp_st(dgo + H + k, dF * fg * (1.f - fg));
      lp_st(dgo + 2 * H + k, dG * (1.f - gg * gg));
      lp_st(dgo + 3 * H + k, dO * og * (1.f - og));
    }
    if (t > 0) lp_publish(sy);
  }
}

__device__ unsigned g_lstm_sync[64][8 * LP_SHARD + 32];   // per (device, stream) slot: shards, error word

// Kernel choice (`kernel` argument: 0 = auto, 1 = the generic kernels, used by tests to pin
// them at shapes the specialised kernels also cover).
// register-resident: one 1024-thread workgroup per clip, W_hh slice in VGPRs
bool lstm_reg(int H, int kernel) { return kernel == 0 && (H == 128 || H == 64); }
// per-step kernels: H = 32 * KS for the instantiated KS, clips within the register partials
bool lstm_step(int B, int H, int kernel) {
  const size_t fwd_lds = ((size_t)B * 32 * (H / 32 + 4) + 8 * B) * sizeof(float);
  const size_t bwd_lds = ((size_t)8 * H + 64 + 2 * B) * sizeof(float);
  return kernel == 0 && !lstm_reg(H, kernel) && (H == 256 || H == 512 || H == 1024) && B <= LS_MAXB &&
         fwd_lds <= 65536 && bwd_lds <= 65536;
}

// persistent kernels for H = 256 / 512, B <= 32, when all G = H / 4 workgroups can be resident at once (the
// occupancy query).  Default: the forward only -- at XceptionLSTMA's shape (B 16, T 120, H 512) it runs 4.6 us
// per step against the per-step kernels' 6.3; the persistent backward (published dh partials) is faster at
// small B (3.9 vs 4.6 us per step at B 2) but slower at B 16 (9.5 vs 7.3: the partials' sc1 traffic), so the
// per-step backward stays there (profiles/r06_lstm_ab.txt); where the clip-grouped backward's workgroups take
// at most half the CUs it is the default (xcp_lstm_bwd).  XCP_LSTM_PERSIST=0: neither, 1: both (read per call).
int lstm_persist_mode() {
  const char* e = getenv("XCP_LSTM_PERSIST");
  return e && e[0] == '0' ? 0 : e && e[0] == '1' ? 2 : 1;
}
bool lstm_persist_env(bool fwd) { return lstm_persist_mode() >= (fwd ? 1 : 2); }
bool lstm_bwd_gather() {   // XCP_LSTM_BWD=gather: the persistent backward's gather form (A/B; read per call)
  const char* e = getenv("XCP_LSTM_BWD");
  return e && e[0] == 'g';
}
int lstm_bwd_cg() {   // XCP_LSTM_BWD=cg / cg2: the clip-grouped gather form, 1 / 2 clips per wave (A/B; read per call)
  const char* e = getenv("XCP_LSTM_BWD");
  if (!(e && e[0] == 'c' && e[1] == 'g')) return 0;
  return e[2] == '2' ? 2 : 1;
}
bool lstm_cg_default(int B, int H, int kernel) {
  return kernel == 0 && B <= 32 && (H == 256 || H == 512) && lstm_persist_mode() == 1 && !getenv("XCP_LSTM_BWD");
}
int lp_cus() {
  static const int v = [] {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      return 0;
    return n;
  }();
  return v;
}
template <typename K>
bool lp_resident(K kern, int G) {
  int dev = 0, cus = 0, per = 0;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    return false;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, kern, 256, 0) != hipSuccess) return false;
  return (long)per * cus >= G;
}
bool lstm_persist(int B, int H, int kernel, bool fwd) {
  if (kernel != 0 || B > 32 || !(H == 256 || H == 512) || !lstm_persist_env(fwd)) return false;
  static int ok[2][2] = {{-1, -1}, {-1, -1}};   // [fwd][H == 512]
  int& v = ok[fwd][H == 512];
  if (v < 0) {
    if (fwd) v = H == 512 ? lp_resident(lstm_fwd_persist_kernel<512>, H / LP_U) : lp_resident(lstm_fwd_persist_kernel<256>, H / LP_U);
    else v = H == 512 ? lp_resident(lstm_bwd_persist_kernel<512>, H / LP_U) : lp_resident(lstm_bwd_persist_kernel<256>, H / LP_U);
  }
  return v == 1;
}

// the sync words of (device, stream), zeroed on the stream before each persistent launch
int lp_sync(hipStream_t st, LstmSync& sy) {
  static std::mutex mu;
  static std::vector<std::pair<int, hipStream_t>> slots;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return XCP_EINVAL;
  int slot = -1;
  {
    std::lock_guard<std::mutex> lk(mu);
    for (size_t i = 0; i < slots.size(); ++i)
      if (slots[i].first == dev && slots[i].second == st) slot = (int)i;
    if (slot < 0) {
      if (slots.size() >= 64) return XCP_EUNSUPPORTED;
      slots.emplace_back(dev, st);
      slot = (int)slots.size() - 1;
    }
  }
  void* base = nullptr;
  if (hipGetSymbolAddress(&base, HIP_SYMBOL(g_lstm_sync)) != hipSuccess) return XCP_EINVAL;
  unsigned* words = reinterpret_cast<unsigned*>(base) + (long)slot * (8 * LP_SHARD + 32);
  if (hipMemsetAsync(words, 0, 8 * LP_SHARD * sizeof(unsigned), st) != hipSuccess) return XCP_EINVAL;
  sy.cnt = words;
  sy.err = words + 8 * LP_SHARD;
  return XCP_OK;
}

}  // namespace


extern "C" {

// 1 when a persistent LSTM launch on any stream gave up waiting for its workgroups (its results are
// invalid); clears the flags.  Synchronises the device.
int xcp_lstm_sync_error() {
  void* base = nullptr;
  if (hipDeviceSynchronize() != hipSuccess || hipGetSymbolAddress(&base, HIP_SYMBOL(g_lstm_sync)) != hipSuccess)
    return -1;
  static unsigned host[64][8 * LP_SHARD + 32];
  if (hipMemcpy(host, base, sizeof(host), hipMemcpyDeviceToHost) != hipSuccess) return -1;
  int any = 0;
  for (int i = 0; i < 64; ++i)
    if (host[i][8 * LP_SHARD]) {
      any = 1;
      unsigned* w = reinterpret_cast<unsigned*>(base) + (long)i * (8 * LP_SHARD + 32) + 8 * LP_SHARD;
      if (hipMemset(w, 0, sizeof(unsigned)) != hipSuccess) return -1;
    }
  return any;
}

// 1 when xcp_lstm_fwd (same B, H, kernel) runs the generic kernel, which reads the transposed W_hh
int xcp_lstm_needs_whhT(int B, int H, int kernel) {
  // (the register-resident, persistent and per-step forward kernels read W_hh as stored)
  return lstm_reg(H, kernel) || lstm_persist(B, H, kernel, true) || lstm_step(B, H, kernel) ? 0 : 1;
}

int xcp_lstm_fwd(const float* xproj, const float* whh, const float* whhT, const float* bih, const float* bhh, float* out,
                 float* hprev, float* cst, float* gates, float* hn, float* cn, int B, int T, int H, int kernel,
                 hipStream_t st) {
  if (B <= 0 || T <= 0) return XCP_OK;
  if (kernel < 0 || kernel > 1) return XCP_EINVAL;
  if (lstm_reg(H, kernel)) {
    if (H == 128)
      hipLaunchKernelGGL(lstm_fwd_reg_kernel<128>, dim3(B), dim3(1024), 0, st, xproj, whh, bih, bhh, out, hprev, cst,
                         gates, hn, cn, T);
    else
      hipLaunchKernelGGL(lstm_fwd_reg_kernel<64>, dim3(B), dim3(1024), 0, st, xproj, whh, bih, bhh, out, hprev, cst,
                         gates, hn, cn, T);
    return (int)hipGetLastError();
  }
  if (lstm_persist(B, H, kernel, true)) {
    LstmSync sy;
    const int rc = lp_sync(st, sy);
    if (rc != XCP_OK) return rc;
    if (H == 512)
      hipLaunchKernelGGL(lstm_fwd_persist_kernel<512>, dim3(H / LP_U), dim3(256), 0, st, xproj, whh, bih, bhh, out, hprev,
                         cst, gates, hn, cn, B, T, sy);
    else
      hipLaunchKernelGGL(lstm_fwd_persist_kernel<256>, dim3(H / LP_U), dim3(256), 0, st, xproj, whh, bih, bhh, out, hprev,
                         cst, gates, hn, cn, B, T, sy);
    return (int)hipGetLastError();
  }
  if (lstm_step(B, H, kernel)) {
    const size_t smem = ((size_t)B * 32 * (H / 32 + 4) + 8 * B) * sizeof(float);
    for (int t = 0; t < T; ++t) {
      if (H == 256)
        hipLaunchKernelGGL(lstm_fwd_step_kernel<8>, dim3(H / LS_UPW), dim3(256), smem, st, xproj, whh, bih, bhh, out,
                           hprev, cst, gates, hn, cn, B, T, t);
      else if (H == 512)
        hipLaunchKernelGGL(lstm_fwd_step_kernel<16>, dim3(H / LS_UPW), dim3(256), smem, st, xproj, whh, bih, bhh, out,
                           hprev, cst, gates, hn, cn, B, T, t);
      else
        hipLaunchKernelGGL(lstm_fwd_step_kernel<32>, dim3(H / LS_UPW), dim3(256), smem, st, xproj, whh, bih, bhh, out,
                           hprev, cst, gates, hn, cn, B, T, t);
    }
    return (int)hipGetLastError();
  }
  if (!whhT) return XCP_EINVAL;
  const size_t smem = (size_t)6 * H * sizeof(float);
  hipLaunchKernelGGL(lstm_fwd_kernel, dim3(B), dim3(256), smem, st, xproj, whhT, bih, bhh, out, hprev, cst, gates, hn, cn,
                     T, H);
  return (int)hipGetLastError();
}

int xcp_lstm_bwd(const float* dout, const float* dhn, const float* dcn, const float* whh, const float* cst,
                 const float* gates, float* dgates, float* work, int B, int T, int H, int kernel, hipStream_t st) {
  if (B <= 0 || T <= 0) return XCP_OK;
  if (kernel < 0 || kernel > 1) return XCP_EINVAL;
  // clip-grouped form: cpw clips per wave, H / 4 x ceil(B / (4 cpw)) workgroups, if they can all be resident
  auto cg_grid = [&](int cpw) { return (H / LP_U) * ((B + 4 * cpw - 1) / (4 * cpw)); };
  auto cg_fits = [&](int cpw) {
    const int g = cg_grid(cpw);
    if (cpw == 1) return H == 512 ? lp_resident(lstm_bwd_cg_kernel<512, 1>, g) : lp_resident(lstm_bwd_cg_kernel<256, 1>, g);
    return H == 512 ? lp_resident(lstm_bwd_cg_kernel<512, 2>, g) : lp_resident(lstm_bwd_cg_kernel<256, 2>, g);
  };
  auto launch_cg = [&](int cpw) {
    LstmSync sy;
    const int rc = lp_sync(st, sy);
    if (rc != XCP_OK) return rc;
    const dim3 g(cg_grid(cpw));
#define XCP_LCG(HH, C) hipLaunchKernelGGL((lstm_bwd_cg_kernel<HH, C>), g, dim3(256), 0, st, dout, dhn, dcn, whh, cst, gates, dgates, B, T, sy)
    if (H == 512 && cpw == 1) XCP_LCG(512, 1);
    else if (H == 512) XCP_LCG(512, 2);
    else if (cpw == 1) XCP_LCG(256, 1);
    else XCP_LCG(256, 2);
#undef XCP_LCG
    return (int)hipGetLastError();
  };
  // default (XCP_LSTM_PERSIST and XCP_LSTM_BWD unset): the clip-grouped persistent backward where its workgroups
  // take at most half the CUs, as the persistent forward's do (H = 512 up to 4 clips, H = 256 up to 8): 30-47 %
  // faster than the per-step kernels there.  Elsewhere the per-step kernels: at XceptionLSTMA's B 16 x H 512 the
  // two-clips-per-wave form (XCP_LSTM_BWD=cg2) is 2 % faster but needs every CU resident at once
  // (profiles/r06_lstm_cg_ab.txt)
  if (lstm_cg_default(B, H, kernel) && 2 * cg_grid(1) <= lp_cus() && cg_fits(1)) return launch_cg(1);
  if (lstm_persist(B, H, kernel, false)) {
    const int cpw = lstm_bwd_cg();
    if (cpw && cg_fits(cpw)) return launch_cg(cpw);
    LstmSync sy;
    const int rc = lp_sync(st, sy);
    if (rc != XCP_OK) return rc;
    if (lstm_bwd_gather()) {
      if (H == 512)
        hipLaunchKernelGGL(lstm_bwd_gather_kernel<512>, dim3(H / LP_U), dim3(256), 0, st, dout, dhn, dcn, whh, cst, gates,
                           dgates, B, T, sy);
      else
        hipLaunchKernelGGL(lstm_bwd_gather_kernel<256>, dim3(H / LP_U), dim3(256), 0, st, dout, dhn, dcn, whh, cst, gates,
                           dgates, B, T, sy);
      return (int)hipGetLastError();
    }
    if (!work) return XCP_EINVAL;
    if (H == 512)
      hipLaunchKernelGGL(lstm_bwd_persist_kernel<512>, dim3(H / LP_U), dim3(256), 0, st, dout, dhn, dcn, whh, cst, gates,
                         dgates, work, B, T, sy);
    else
      hipLaunchKernelGGL(lstm_bwd_persist_kernel<256>, dim3(H / LP_U), dim3(256), 0, st, dout, dhn, dcn, whh, cst, gates,
                         dgates, work, B, T, sy);
    return (int)hipGetLastError();
  }
  if (lstm_step(B, H, kernel)) {
    if (!work) return XCP_EINVAL;
    float* whhT = work + (long)B * H;
    hipLaunchKernelGGL(lstm_transpose_kernel, dim3(4 * H / 32, H / 32), dim3(256), 0, st, whh, whhT, H);
    const size_t smem = ((size_t)8 * H + 64 + 2 * B) * sizeof(float);
    for (int t = T - 1; t >= 0; --t)
      hipLaunchKernelGGL(lstm_bwd_step_kernel, dim3(H / LS_UPW), dim3(256), smem, st, dout, dhn, dcn, whhT, cst, gates,
                         dgates, work, B, T, H, t);
    return (int)hipGetLastError();
  }
  if (lstm_reg(H, kernel)) {
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
