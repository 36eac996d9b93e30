// Fused backward of one narrow SeparableConv2d + BatchNorm2d unit: the entry-flow units of
// block1 (147^2: 64 -> 128, 128 -> 128 channels) and block2 (74^2: 128 -> 256, 256 -> 256),
// Xception.py:61-87.
//
// Given, per pixel row m, the gradient G[m][co] w.r.t. the BN output, the BN input Y[m][co]
// (= the pointwise output) and the BN-backward coefficients (alpha, bcoef, delta) of that BN
// (from its finalised batch sums), one pass computes
//   dY[m][co] = bf16(alpha[co] * G + (bcoef[co] * Y + delta[co]))   (as bn_bwd_apply_kernel)
//   dD[m][ci] = sum_co dY[m][co] * W[co][ci]                           (pointwise dgrad)
//   P[s][co][ci] = sum_{m in split s} dY[m][co] * X[m][ci]            (pointwise wgrad slabs)
// so dY never goes to HBM: the unfused sequence (bn_bwd_apply, gemm_nt dgrad, gemm_tn wgrad)
// reads G, Y once and dY twice, writes dY once; this reads G, Y, X and writes dD only.
// HBM-bound: bytes per pixel row = 2*(2*CO + 2*CI) (bf16).
//
// Workgroup = 4 or 8 waves over one row split (and one block of 128 input channels when
// CI = 256), 64-row tiles: the next tile's G / Y / X rows are loaded into registers while the
// current tile's MFMAs run; dY and X are staged in LDS ([m][c], 8 (mod 64)-dword pitches so the
// transposed ds_read_b64_tr_b16 fragment reads of the weight gradient are conflict-free), the
// block's rows of W^T stay in LDS for the whole split, and dD is transposed through LDS for
// 16-B stores.
#include "common.h"

namespace {

constexpr int UB_TM = 64;                  // pixel rows per tile

struct UnitBwdArgs {
  const bf16* G;       // [M][CO] gradient w.r.t. the BN output
  const bf16* Y;       // [M][CO] BN input (pointwise output)
  const float* alpha;  // [CO]
  const float* bcoef;  // [CO]
  const float* delta;  // [CO]
  const bf16* Wt;      // [CI][CO] pointwise weight, transposed (engine's pwT pack)
  const bf16* X;       // [M][CI] pointwise input (depthwise output)
  bf16* dD;            // [M][CI] gradient w.r.t. the pointwise input
  float* P;            // [S][CO][CI] weight-gradient partial slabs
  int M, CI, S, rows_per_split;
};

// CO: unit output channels; CIW: input channels per workgroup (grid = S splits x CI / CIW
// channel blocks: the blocks of one split are adjacent ids, so they run together on one XCD
// and the second reads G / Y from L2); NTH: threads.
constexpr int UB_DWORD3 = 0x00020000;   // gfx9 raw buffer descriptor word 3
constexpr int UB_RECORDS = 0x7fffffff;
constexpr int UB_OOB = (int)0x80000000u;   // >= num_records: loads return zeros, stores are dropped
typedef int ub_i32x4 __attribute__((ext_vector_type(4)));

template <int CO, int CIW, int NTH>
__global__ __launch_bounds__(NTH, 512 / NTH) void unit_bwd_kernel(UnitBwdArgs a) {
  constexpr int TM = UB_TM;
  constexpr int NW = NTH / 64;               // waves
  constexpr int DP = CO * 2 + 32;            // sD pitch (bytes): 8 (mod 64) dwords, conflict-free tr reads
  constexpr int WP = CO * 2 + 16;            // sW pitch: 4 (mod 64) dwords, conflict-free b128 rows
  constexpr int XP = CIW * 2 + 32;           // sX / sOut pitch
  constexpr int GCH = CO / 8;                // 16-B chunks per G / Y row
  constexpr int GLD = TM * GCH / NTH;        // G (and Y) chunks per thread per tile
  constexpr int XCH = CIW / 8;               // 16-B chunks per X row (this block's channels)
  constexpr int XLD = TM * XCH / NTH;        // X chunks per thread per tile
  constexpr int WMS = CO / 64;               // wgrad: waves along co (64 each) ...
  constexpr int WNS = NW / WMS;              // ... and along ci
  constexpr int WN = CIW / WNS;              // wgrad wave tile: 64 co x WN ci
  constexpr int NJ = WN / 16;
  constexpr int DCI = CIW / NW;              // dgrad wave tile: DCI ci x 64 m
  constexpr int NDI = DCI / 16;
  static_assert(NTH % GCH == 0 && NTH % XCH == 0 && GLD >= 1 && XLD >= 1, "load mapping");
  static_assert(WMS * WNS == NW && NJ >= 1 && NDI >= 1, "wave tiling");
  __shared__ __attribute__((aligned(16))) char sW[CIW * WP];
  __shared__ __attribute__((aligned(16))) char sD[TM * DP];
  __shared__ __attribute__((aligned(16))) char sX[TM * XP];

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int fr = lane & 15, fg = lane >> 4, q4 = fr >> 2, p4 = fr & 3;
  const int nblk = a.CI / CIW;
  const int id = xcd_remap(blockIdx.x, gridDim.x);
  const int s = id / nblk, c0 = (id % nblk) * CIW;   // split, first input channel of this block
  const long mbeg = (long)s * a.rows_per_split;
  const long mend = min((long)a.M, mbeg + a.rows_per_split);
  if (mbeg >= mend) return;   // (the host sizes S so that every split has rows)

  // this block's rows of W^T -> LDS once
  for (int q = tid; q < CIW * GCH; q += NTH) {
    const int r = q / GCH, c = q % GCH;
    *reinterpret_cast<uint4*>(sW + r * WP + c * 16) =
        *reinterpret_cast<const uint4*>(a.Wt + (long)(c0 + r) * CO + c * 8);
  }
  // this thread's G / Y chunk column is fixed: channels 8*gc .. 8*gc+7
  const int gc = tid % GCH, grow = tid / GCH;   // rows grow + (NTH / GCH) i
  float al[8], bc[8], de[8];
  VecIO<float, 8>::load(a.alpha + gc * 8, al);
  VecIO<float, 8>::load(a.bcoef + gc * 8, bc);
  VecIO<float, 8>::load(a.delta + gc * 8, de);
  const int xc = tid % XCH, xrow = tid / XCH;   // X rows xrow + (NTH / XCH) i

  // G, Y, X and dD through buffer resources on this split's rows: 32-bit offsets from the split's first
  // row, the per-thread part fixed, rows past the split out of range (loads return zeros -- stage_tile
  // masks those rows anyway -- and stores are dropped).  (The 64-bit row products per load and store
  // were a fifth of the kernel's VALU.)
  // (num_records is the 2 GB maximum -- the GEMMs measured an exact span slower -- and rows past the
  // split get the out-of-range offset explicitly)
  const int nrows = (int)(mend - mbeg);
  const __amdgpu_buffer_rsrc_t rsG = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16*>(a.G + mbeg * CO), (short)0,
                                                                       UB_RECORDS, UB_DWORD3);
  const __amdgpu_buffer_rsrc_t rsY = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16*>(a.Y + mbeg * CO), (short)0,
                                                                       UB_RECORDS, UB_DWORD3);
  const __amdgpu_buffer_rsrc_t rsX = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16*>(a.X + mbeg * a.CI), (short)0,
                                                                       UB_RECORDS, UB_DWORD3);
  const int goff = (grow * CO + gc * 8) * 2, xoff = (xrow * a.CI + c0 + xc * 8) * 2;
  uint4 rG[GLD], rY[GLD], rX[XLD];
  auto load_tile = [&](long m0) {
    const int tb = (int)(m0 - mbeg);   // tile's first row within the split
#pragma unroll
    for (int i = 0; i < GLD; ++i) {
      const int rw = tb + grow + (NTH / GCH) * i;
      const int o = rw < nrows ? (tb + (NTH / GCH) * i) * CO * 2 + goff : UB_OOB;
      rG[i] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rsG, o, 0, 0));
      rY[i] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rsY, o, 0, 0));
    }
#pragma unroll
    for (int i = 0; i < XLD; ++i) {
      const int rw = tb + xrow + (NTH / XCH) * i;
      rX[i] = __builtin_bit_cast(
          uint4, __builtin_amdgcn_raw_buffer_load_b128(rsX, rw < nrows ? (tb + (NTH / XCH) * i) * a.CI * 2 + xoff : UB_OOB, 0, 0));
    }
  };
  auto stage_tile = [&](long m0) {
#pragma unroll
    for (int i = 0; i < GLD; ++i) {
      const int r = grow + (NTH / GCH) * i;
      float g[8], y[8];
      VecIO<bf16, 8>::load(reinterpret_cast<const bf16*>(&rG[i]), g);
      VecIO<bf16, 8>::load(reinterpret_cast<const bf16*>(&rY[i]), y);
      const bool ok = m0 + r < mend;   // rows past the split: dY = 0 (not delta)
#pragma unroll
      for (int j = 0; j < 8; ++j) g[j] = ok ? fmaf(al[j], g[j], fmaf(bc[j], y[j], de[j])) : 0.f;
      VecIO<bf16, 8>::store(reinterpret_cast<bf16*>(sD + r * DP + gc * 16), g);
    }
#pragma unroll
    for (int i = 0; i < XLD; ++i) {
      const int r = xrow + (NTH / XCH) * i;
      *reinterpret_cast<uint4*>(sX + r * XP + xc * 16) = m0 + r < mend ? rX[i] : make_uint4(0, 0, 0, 0);
    }
  };

  const __amdgpu_buffer_rsrc_t rsD = __builtin_amdgcn_make_buffer_rsrc(a.dD + mbeg * a.CI, (short)0, UB_RECORDS, UB_DWORD3);
  f32x4 accw[4][NJ];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) accw[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int wm = w / WNS, wn = w % WNS;   // wgrad wave tile: co wm*64.., ci wn*WN..

  load_tile(mbeg);
  for (long m0 = mbeg; m0 < mend; m0 += TM) {
    lds_barrier();            // previous tile's readers of sD / sX (sOut) are done
    stage_tile(m0);
    lds_barrier();
    if (m0 + TM < mend) load_tile(m0 + TM);

    // weight gradient: accw += dY^T X over the tile's 64 rows (2 MFMA k-steps of 32 rows)
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 af[4], bfr[NJ];
#pragma unroll
      for (int t4 = 0; t4 < 4; ++t4) {
        const int ncol = wm * 64 + t4 * 16 + p4 * 4;
        const bf16x4 a0 = ds_read_tr(sD + (32 * ks + 4 * fg + q4) * DP + ncol * 2);
        const bf16x4 a1 = ds_read_tr(sD + (32 * ks + 16 + 4 * fg + q4) * DP + ncol * 2);
        af[t4] = bf16x8{a0[0], a0[1], a0[2], a0[3], a1[0], a1[1], a1[2], a1[3]};
      }
#pragma unroll
      for (int t4 = 0; t4 < NJ; ++t4) {
        const int kcol = wn * WN + t4 * 16 + p4 * 4;
        const bf16x4 b0 = ds_read_tr(sX + (32 * ks + 4 * fg + q4) * XP + kcol * 2);
        const bf16x4 b1 = ds_read_tr(sX + (32 * ks + 16 + 4 * fg + q4) * XP + kcol * 2);
        bfr[t4] = bf16x8{b0[0], b0[1], b0[2], b0[3], b1[0], b1[1], b1[2], b1[3]};
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j) accw[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], accw[i][j], 0, 0, 0);
    }

    // dgrad, transposed: dD^T[ci][m] = sum_co W^T[ci][co] dY[m][co]; wave w: ci w*DCI.., all 64 m
    f32x4 accd[NDI][4];
#pragma unroll
    for (int i = 0; i < NDI; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) accd[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int k0 = 0; k0 < CO; k0 += 32) {
      bf16x8 wa[NDI], db[4];
#pragma unroll
      for (int i = 0; i < NDI; ++i)
        wa[i] = *reinterpret_cast<const bf16x8*>(sW + (w * DCI + i * 16 + fr) * WP + (k0 + 8 * fg) * 2);
#pragma unroll
      for (int j = 0; j < 4; ++j)
        db[j] = *reinterpret_cast<const bf16x8*>(sD + (j * 16 + fr) * DP + (k0 + 8 * fg) * 2);
#pragma unroll
      for (int i = 0; i < NDI; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) accd[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa[i], db[j], accd[i][j], 0, 0, 0);
    }
    lds_barrier();            // every wave is done reading sX (weight gradient)
    // accd[i][j][r] = dD[m = j*16 + fr][ci = w*DCI + i*16 + 4*fg + r] -> sOut (= sX) as bf16
#pragma unroll
    for (int i = 0; i < NDI; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        bf16x4 q;
#pragma unroll
        for (int r = 0; r < 4; ++r) q[r] = (bf16)accd[i][j][r];
        *reinterpret_cast<bf16x4*>(sX + (j * 16 + fr) * XP + (w * DCI + i * 16 + 4 * fg) * 2) = q;
      }
    lds_barrier();
#pragma unroll
    for (int i = 0; i < XLD; ++i) {
      const int r = xrow + (NTH / XCH) * i;
      const int rw = (int)(m0 - mbeg) + r;
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(ub_i32x4, *reinterpret_cast<const uint4*>(sX + r * XP + xc * 16)),
                                             rsD, rw < nrows ? ((int)(m0 - mbeg) + (NTH / XCH) * i) * a.CI * 2 + xoff : UB_OOB, 0, 0);
    }
  }
  // weight-gradient slab: accw[i][j][r] = P[co = wm*64 + i*16 + 4*fg + r][ci = c0 + wn*WN + j*16 + fr]
  float* P = a.P + (long)s * CO * a.CI + c0;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int j = 0; j < NJ; ++j)
        P[(long)(wm * 64 + i * 16 + 4 * fg + r) * a.CI + wn * WN + j * 16 + fr] = accw[i][j][r];
}

// supported shapes: (CO, CI) -> input channels per block and target row splits
// (CO 128: 2 workgroups of 256 threads per CU, 512 splits; CO 256: one of 512 per CU,
// CI / 128 blocks per split, 256 workgroups)
bool unit_cfg(int CO, int CI, int& ciw, int& splits) {
  if (CO == 128 && (CI == 64 || CI == 128)) {
    ciw = CI;
    splits = 512;
    return true;
  }
  if (CO == 256 && (CI == 128 || CI == 256)) {
    ciw = 128;
    splits = 256 / (CI / 128);
    return true;
  }
  return false;
}

}  // namespace

extern "C" {

// rows per split of xcp_unit_bwd (0: shape not supported by the fused kernel)
int xcp_unit_bwd_rows_per_split(int dtype, int M, int CO, int CI) {
  int ciw, splits;
  if (dtype != XCP_BF16 || M <= 0 || !unit_cfg(CO, CI, ciw, splits)) return 0;
  const long per = ((long)M + splits - 1) / splits;
  return (int)((per + UB_TM - 1) / UB_TM * UB_TM);
}

int xcp_unit_bwd(int dtype, const void* G, const void* Y, const float* alpha, const float* bcoef, const float* delta,
                 const void* Wt, const void* X, void* dD, float* P, int M, int CO, int CI, int S, int rows_per_split,
                 hipStream_t stream) {
  if (M <= 0) return XCP_OK;
  const int rps = xcp_unit_bwd_rows_per_split(dtype, M, CO, CI);
  if (rps == 0) return XCP_EUNSUPPORTED;
  if (rows_per_split != rps || S != (M + rps - 1) / rps) return XCP_EINVAL;
  UnitBwdArgs a{(const bf16*)G, (const bf16*)Y, alpha, bcoef, delta, (const bf16*)Wt, (const bf16*)X, (bf16*)dD,
                P, M, CI, S, rows_per_split};
  const dim3 grid(S * (CO == 256 ? CI / 128 : 1));
  if (CO == 128 && CI == 128) hipLaunchKernelGGL((unit_bwd_kernel<128, 128, 256>), grid, dim3(256), 0, stream, a);
  else if (CO == 128) hipLaunchKernelGGL((unit_bwd_kernel<128, 64, 256>), grid, dim3(256), 0, stream, a);
  else hipLaunchKernelGGL((unit_bwd_kernel<256, 128, 512>), grid, dim3(512), 0, stream, a);
  return (int)hipGetLastError();
}

}  // extern "C"
