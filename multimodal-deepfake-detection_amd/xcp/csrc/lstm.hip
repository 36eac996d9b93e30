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

}  // namespace


extern "C" {

// 1 when xcp_lstm_fwd (same B, H, kernel) runs the generic kernel, which reads the transposed W_hh
int xcp_lstm_needs_whhT(int B, int H, int kernel) { return lstm_reg(H, kernel) || lstm_step(B, H, kernel) ? 0 : 1; }

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
