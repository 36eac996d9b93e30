/* xcp.h -- C ABI of the MI355X-native Xception + LSTM clip-classification path.
 *
 * Drop-in boundary for the hot path of Tonmoy1321/Multimodal-DeepFake-Detection:
 * the Xception entry/middle/exit-flow SeparableConv2d stacks (Xception.py:37-201)
 * and the per-clip LSTM of XceptionLSTMV / XceptionLSTMA (XceptionLSTMV.py:18-23,
 * :66-70; XceptionLSTMA.py:14-19, :55-59).  The reference binds to these ops only
 * implicitly, through torch.nn modules; the host mirror
 * (multimodal-deepfake-detection_amd/Models, .../xcp) binds each entry point below
 * with ctypes.
 *
 * Conventions (every entry point):
 *  - plain device pointers and sizes; pointers are never freed or retained;
 *  - activations are NHWC "pixel rows" of C channels; `dtype` selects the storage
 *    type of activation / GEMM operands: 0 = fp32 (parity mode), 1 = bf16;
 *    accumulation is fp32, BN statistics fp64, master weights / grads fp32;
 *  - work is enqueued on `stream` (a hipStream_t) with no host synchronisation and
 *    no allocation, so a caller may capture it into a hipGraph;
 *  - return 0 on success, a hipError_t code, or XCP_EINVAL (1001) /
 *    XCP_EUNSUPPORTED (1002).  No C++ exception crosses the ABI.
 */
#ifndef XCP_H_
#define XCP_H_

#ifdef __cplusplus
extern "C" {
#endif

typedef void* xcp_stream_t; /* hipStream_t */

#define XCP_OK 0
#define XCP_EINVAL 1001
#define XCP_EUNSUPPORTED 1002
#define XCP_F32 0
#define XCP_BF16 1
#define XCP_ACT_NONE 0
#define XCP_ACT_RELU 1
#define XCP_ACT_BNRELU 2

/* ---- pointwise 1x1 conv / skip conv / stem conv2 / LSTM input projection ----
 * replaces nn.Conv2d(C, Cout, 1) of SeparableConv2d.pointwise (Xception.py:42,:46),
 * Block.skip (Xception.py:55,:93), Xception.conv2 (Xception.py:122,:172; im2col
 * gather mode 2, its input gradient via mode 3) and x @ W_ih^T of nn.LSTM.
 * C[M,N] = A[M,K] . B[N,K]^T ; optional stats[xcp_gemm_nt_stat_rows(M)][2][N] partial
 * (sum, sum^2) of the stored C columns (BatchNorm batch statistics).
 * gmode: 0 dense rows, 1 strided (skip conv, stride gS), 2 im2col 3x3 p0,
 *        3 transposed im2col (conv input gradient); gC = channels per tap.
 * tile: 0 = automatic (256x256 8-wave kernel for dense bf16 with >= 256 output tiles and
 *       K >= 384, or outputs >= 256 wide and K >= 128 -- its persistent form, one workgroup
 *       per CU walking the tiles, with a less than 3/4 full last round of tiles sent to the
 *       128x128 kernel -- else 128x128), 1 = force 128x128, 2 = force the one-shot 256x256
 *       for every row, 3 = force the persistent 256x256 for every row (dense bf16 only),
 *       4 = automatic with the one-shot 256x256 kernel. */
int xcp_gemm_nt(int dtype, const void* A, long lda, const void* B, long ldb, void* C, long ldc, int M, int N, int K,
                float* stats, int gmode, int gH, int gW, int gOH, int gOW, int gS, int gC, int tile, xcp_stream_t stream);
/* number of partial rows in gemm_nt's stats array for M rows */
int xcp_gemm_nt_stat_rows(int M);

/* weight gradient of the above: P[s][N][K] = sum_{m in split s} G[m][N] X[m][K],
 * rows split in S chunks of rows_per_split; X rows gathered as in gemm_nt
 * (gmode 0-2).  Reduce P over s with xcp_colreduce_f32.  tile: 0 automatic (256x256 for
 * dense bf16 with N, K >= 256), 1 = 128x128, 2 = 256x256; pass the same value to both calls. */
/* rows per split to pass to xcp_gemm_tn for this problem (S = ceil(M / rows)). */
int xcp_gemm_tn_rows_per_split(int dtype, int gmode, int M, int N, int K, int tile);
int xcp_gemm_tn(int dtype, const void* G, long ldg, const void* X, long ldx, float* P, int M, int N, int K, int S,
                int rows_per_split, int gmode, int gH, int gW, int gOH, int gOW, int gS, int gC, int tile,
                xcp_stream_t stream);

/* fused backward of one SeparableConv2d's pointwise conv + its BatchNorm2d (Xception.py:44-47
 * then :56/:67/:73/:78 BN; replaces xcp_bn_bwd_apply + xcp_gemm_nt dgrad + xcp_gemm_tn wgrad for
 * the unit): dY = alpha*G + (bcoef*Y + delta) (bf16-rounded, never stored),
 * dD[M][CI] = dY Wt^T, P[s][CO][CI] = sum_{m in split s} dY[m][co] X[m][ci] (reduce with
 * xcp_colreduce_f32).  Wt: [CI][CO].  bf16; (CO, CI) = (128, 64 | 128) or (256, 128 | 256) only. */
/* rows per split (S = ceil(M / rows)); 0: the shape is not supported */
int xcp_unit_bwd_rows_per_split(int dtype, int M, int CO, int CI);
int xcp_unit_bwd(int dtype, const void* G, const void* Y, const float* alpha, const float* bcoef, const float* delta,
                 const void* Wt, const void* X, void* dD, float* P, int M, int CO, int CI, int S, int rows_per_split,
                 xcp_stream_t stream);

/* ---- depthwise 3x3 (SeparableConv2d.conv1, Xception.py:41,:45) ----
 * Y = dw3x3(act(X)); act per XCP_ACT_* (BN scale/shift for XCP_ACT_BNRELU);
 * Wt is the [9][C] fp32 tap-major packing of the [C,1,3,3] weight. */
int xcp_dw_fwd(int dtype, int act, const void* X, void* Y, const float* Wt, const float* scale, const float* shift, int N,
               int H, int W, int C, xcp_stream_t stream);
/* fused depthwise + pointwise forward of an entry-flow unit (Xception.py:37-47; block1's units, block2's first):
 * D = dw3x3(act(X)) (bitwise xcp_dw_fwd's), Y = D . pw^T (bitwise xcp_gemm_nt's),
 * part[R][2][COUT] BN partial sums (sum, sum of squares) of the stored bf16 Y, R = xcp_sep_fwd_parts().
 * dwt: [9][CIN] fp32 taps; pw: [COUT][CIN] bf16.  bf16; (CIN, COUT) = (64 | 128, 128) with W <= 152 or
 * (128, 256) with W <= 78. */
int xcp_sep_fwd_parts(int dtype, int N, int H, int W, int CIN, int COUT);   /* 0: shape not supported */
int xcp_sep_fwd(int dtype, int act, const void* X, const float* scale, const float* shift, const float* dwt, const void* pw,
                void* D, void* Y, float* part, int N, int H, int W, int CIN, int COUT, xcp_stream_t stream);
/* fused backward: dX = act'(X) * dgrad(dY) + dRes + scatter_stride(dSkip) (skip_pre = 0), or
 * act'(X) * (dgrad(dY) + scatter_stride(dSkip)) + dRes (skip_pre = 1: the strided skip conv read the
 * same activation act(X), so its gradient passes the mask and enters the BN partial sums);
 * dWpart[P][C][9] workgroup partials of the weight gradient, P = xcp_dw_bwd_chunks();
 * optional bnpart[P][2][C] = (sum dX, sum dX*(X-bmean)*binvstd): the backward
 * partial sums of the BatchNorm that produced X (XCP_ACT_BNRELU only). */
int xcp_dw_bwd_chunks(int N, int H, int W, int C);
int xcp_dw_bwd(int dtype, int act, const void* dY, const void* X, const float* Wt, const float* scale, const float* shift,
               const void* dRes, const void* dSkip, int sOH, int sOW, int sS, int skip_pre, void* dX, float* dWpart,
               float* bnpart, const float* bmean, const float* binvstd, int N, int H, int W, int C,
               xcp_stream_t stream);
/* The same backward with a residual input dRes (no skip input) whose BatchNorm partial sums are
 * those of the BN whose OUTPUT gradient is the final dX = act'(X) * dA + dRes (an identity-skip block
 * boundary, Xception.py:89-99 (skip = inp, x += skip at :96-98): the previous block's last BN feeds both this block's first ReLU and its
 * residual add): bnpart[P][2][C] = (sum dX, sum dX * (Yb - bmean) * binvstd), dX as stored, Yb that
 * BN's input.  Replaces the separate per-channel reduce of the backward for that BN. */
int xcp_dw_bwd_resbn(int dtype, int act, const void* dY, const void* X, const float* Wt, const float* scale,
                     const float* shift, const void* dRes, void* dX, float* dWpart, float* bnpart, const float* bmean,
                     const float* binvstd, const void* Yb, int N, int H, int W, int C, xcp_stream_t stream);

/* ---- BatchNorm2d (Xception.py:56,67,73,78,119,123,143,147), tails, pooling ---- */
/* out[g][l] = sum over the g-th of G contiguous groups of slabs s of in[s*ld + l], l < L <= ld
 * (fp64 sums, fp32 out); accumulate = 1 (G = 1 only): out[l] += that sum (gradient accumulation
 * into param.grad) */
int xcp_colreduce_f32(const float* in, int S, long L, long ld, float* out, int G, int accumulate, xcp_stream_t stream);
/* up to 16 column reductions in one launch: jobs = HOST int64 [njobs][7] = (in, out, S, L, ld, G,
 * accumulate), each as xcp_colreduce_f32 (bitwise the same outputs); L, ld multiples of 4, in /
 * out 16-B aligned (the backbone backward batches one block's weight-gradient slab reductions) */
int xcp_colreduce_multi(const long long* jobs, int njobs, xcp_stream_t stream);
/* slab groups G for the first level of a two-level reduction of S slabs of L floats (0: one pass) */
int xcp_colreduce_groups(int S, long L);
int xcp_chanred_parts(long rows, int C);
int xcp_row_stats(int dtype, const void* X, long rows, int C, float* part, xcp_stream_t stream);
/* ms / mt (both null, or both set): scale / shift of the BN when dZ is the gradient of
 * relu(bn(Y)) -- the ReLU mask (Y*ms+mt > 0) is applied on the fly (replaces xcp_relu_bwd) */
int xcp_bn_bwd_reduce(int dtype, const void* dZ, const void* Y, const float* mean, const float* invstd,
                      const float* ms, const float* mt, long rows, int C, float* part, xcp_stream_t stream);
/* train-mode finalize straight from fp32 partial rows part[R][2][CP] (sum, sum of squares /
 * sum dz, sum dz*zhat); fp64 accumulation.  C channels of a tensor with channel pitch CP >= C
 * (the padded 736-channel layout of the 728-channel flow): gamma / beta / running stats /
 * dgamma / dbeta have C entries, the per-channel outputs (mean .. shift, alpha .. delta) CP,
 * zero for the padding channels */
int xcp_bn_finalize_part(const float* part, int R, int C, int CP, double count, const float* gamma, const float* beta,
                         float* rmean, float* rvar, float momentum, float eps, float* mean_o, float* invstd_o,
                         float* scale_o, float* shift_o, xcp_stream_t stream);
/* (dgamma, dbeta may be null.)  flags: XCP_FIN_ACCUMULATE adds to dgamma / dbeta (gradient accumulation into
 * param.grad); XCP_FIN_NARROW reduces with 4-wave instead of 16-wave workgroups, which fit beside a kernel
 * that holds every CU (other summation order: same values to fp64 rounding, not the same bits) */
#define XCP_FIN_ACCUMULATE 1
#define XCP_FIN_NARROW 2
int xcp_bn_bwd_finalize_part(const float* part, int R, int C, int CP, double count, const float* gamma,
                             const float* mean, const float* invstd, float* alpha, float* bcoef, float* delta,
                             float* dgamma, float* dbeta, int flags, xcp_stream_t stream);
int xcp_bn_finalize(const double* part2, int G, int C, int CP, double count, const float* gamma, const float* beta,
                    float* rmean, float* rvar, float momentum, float eps, int train, float* mean, float* invstd,
                    float* scale, float* shift, xcp_stream_t stream);
int xcp_bn_act(int dtype, const void* X, void* Y, const float* scale, const float* shift, int relu, long rows, int C,
               xcp_stream_t stream);
/* Y[n][oh][ow][c] = act(X[n][oh*S][ow*S][c] * scale[c] + shift[c]) (relu: max(., 0)): the activated
 * input of a stride-S 1x1 conv (Block.skip, Xception.py:55) when the full-resolution activation is
 * never materialised (its other consumer applies the BN + ReLU on load). */
int xcp_bn_act_strided(int dtype, const void* X, void* Y, const float* scale, const float* shift, int relu, int N, int H,
                       int W, int OH, int OW, int S, int C, xcp_stream_t stream);
int xcp_bn_bwd_apply(int dtype, const void* dZ, const void* Y, void* dY, const float* alpha, const float* bcoef,
                     const float* delta, const float* ms, const float* mt, long rows, int C, xcp_stream_t stream);
int xcp_relu_bwd(int dtype, void* dX, const void* X, long rows, int C, xcp_stream_t stream);
/* Block tail (Xception.py:86,:93-98): Out = [maxpool3x3s2p1](Y*s1+t1) + (s2 ? S*s2+t2 : S) */
int xcp_tail_fwd(int dtype, const void* Y, const float* s1, const float* t1, int pool, const void* S, const float* s2,
                 const float* t2, void* Out, unsigned char* amax, int N, int H, int W, int C, xcp_stream_t stream);
int xcp_maxpool_bwd(int dtype, const void* dOut, const unsigned char* amax, void* dZ, int N, int H, int W, int C,
                    xcp_stream_t stream);
/* xcp_maxpool_bwd fused with the BatchNorm-backward reduce (Xception.py:85-86: the BN before
 * the pool) of its output against Y [N][H][W][C]: part[P][2][C] = per-chunk (sum dz,
 * sum dz*(y-mean)*invstd), P = xcp_maxpool_bwd_bnred_parts(...) */
int xcp_maxpool_bwd_bnred_parts(int N, int H, int W, int C);
int xcp_maxpool_bwd_bnred(int dtype, const void* dOut, const unsigned char* amax, void* dZ, const void* Y,
                          const float* mean, const float* invstd, int N, int H, int W, int C, float* part,
                          xcp_stream_t stream);
/* bn4 + ReLU + adaptive_avg_pool2d (Xception.py:193-198) -> F[N][C] fp32 */
int xcp_avgpool_fwd(int dtype, const void* Y, const float* s, const float* t, float* F, int N, int HW, int C,
                    xcp_stream_t stream);
int xcp_avgpool_bwd(int dtype, const float* dF, const void* Y, const float* s, const float* t, void* dZ, int N, int HW,
                    int C, xcp_stream_t stream);

/* ---- stem conv1 (Xception.py:118,:168) and weight packing ---- */
int xcp_conv1_fwd(int dtype, const float* X, const float* W, void* Y, int N, int IH, int IW, xcp_stream_t stream);
/* conv1 forward + BN1's batch-statistics partials (sum y, sum y^2 of the stored outputs) in
 * part[xcp_conv1_fwd_parts(N, IH, IW)][2][32], for the shapes of xcp_conv1_wgrad_fused (Xception.py:168-169:
 * the partial rows replace a per-channel reduce over the output) */
int xcp_conv1_fwd_parts(int N, int IH, int IW);
int xcp_conv1_fwd_stats(int dtype, const float* X, const float* W, void* Y, float* part, int N, int IH, int IW,
                        xcp_stream_t stream);
int xcp_conv1_wgrad_parts(int N, int IH, int IW);
int xcp_conv1_wgrad(int dtype, const float* X, const void* dY, float* part, int N, int IH, int IW, xcp_stream_t stream);
/* 1 when xcp_conv1_wgrad_bn takes the shape (bf16, frames <= 320 wide), else 0 */
int xcp_conv1_wgrad_fused(int dtype, int IH, int IW);
/* conv1 weight-gradient partials (as xcp_conv1_wgrad) of dC1 = alpha*g + bcoef*Y + delta, formed on load
 * and rounded to the storage type: BN1's backward apply (Xception.py:119,:169; coefficients from
 * xcp_bn_bwd_finalize*), g = dZ masked to 0 where Y*mscale + mshift <= 0 (the ReLU of Xception.py:170)
 * when mscale / mshift are given.  Replaces xcp_bn_bwd_apply + xcp_conv1_wgrad on the stored dC1. */
int xcp_conv1_wgrad_bn(int dtype, const float* X, const void* dZ, const void* Y, const float* alpha, const float* bcoef,
                       const float* delta, const float* mscale, const float* mshift, float* part, int N, int IH, int IW,
                       xcp_stream_t stream);
int xcp_permute3(int out_dtype, const float* in, void* out, int d0, int d1, int d2, int p0, int p1, int p2,
                 xcp_stream_t stream);

/* ---- stem conv2 (Xception.py:122, :172) as a direct MFMA convolution, bf16 ----
 * mode 0: Y[N][IH-2][IW-2][64] = conv3x3(X[N][IH][IW][32], W[64][9][32]); stats (may be null):
 *         BatchNorm partial sums [parts][2][64] of the stored values
 * mode 1: input gradient: Y[N][IH+2][IW+2][32] from X = dY[N][IH][IW][64], W = [32][9][64]
 * in_scale / in_shift (mode 0, may be null): X is the raw input of a BatchNorm + ReLU, applied on load
 * (relu(x * in_scale[c] + in_shift[c]) rounded to bf16: bitwise the xcp_bn_act of X fed in)
 * xcp_conv3x3_parts returns the workgroup count (stats rows), 0 if the width is unsupported */
int xcp_conv3x3_parts(int mode, int N, int IH, int IW);
int xcp_conv3x3(int mode, const void* X, const void* W, void* Y, float* stats, int N, int IH, int IW,
                const float* in_scale, const float* in_shift, xcp_stream_t stream);
/* weight gradient of mode 0 (replaces the autograd wgrad of Xception.conv2, Xception.py:122):
 * P[parts][64][9*32] fp32 slabs whose sum is dW[co][kh*3+kw][ci], from dY[N][IH-2][IW-2][64]
 * and X[N][IH][IW][32]; xcp_conv3x3_wgrad_parts returns the slab count, 0 if unsupported */
int xcp_conv3x3_wgrad_parts(int N, int IH, int IW);
int xcp_conv3x3_wgrad(const void* dY, const void* X, float* P, int N, int IH, int IW, const float* in_scale,
                      const float* in_shift, xcp_stream_t stream);   /* in_scale / in_shift: as xcp_conv3x3 */

/* ---- clip input (video_dataloader.py:22-68): uint8 frames -> fp32 model input ----
 * in [B][Tmax][H][W][3] uint8 (device), len [B] int32 (device): frames t >= len[b] are padding;
 * out [B][Tmax][3][H][W] fp32 = x / 255 (zeros for padding), bit-identical to the host loader;
 * W a multiple of 4 */
int xcp_frames_u8_to_f32(const unsigned char* in, const int* len, float* out, int B, int Tmax, int H, int W,
                         xcp_stream_t stream);

/* ---- clip input, general form: the same x / 255, optionally resized and in the model's layout ----
 * out = F.interpolate(x / 255, (OH, OW), mode="bilinear", align_corners=False) when (OH, OW) !=
 * (H, W) (e.g. the dataset's 256^2 faces -> Xception's 299^2), else x / 255; dtype XCP_F32 or
 * XCP_BF16 (round to nearest even); nhwc 0: [B][Tmax][3][OH][OW], 1: [B][Tmax][OH][OW][3]
 * (channels_last).  Replaces video_dataloader.py:35 + :59-64 (+ the resize a 299^2 run adds). */
int xcp_frames_prep(const unsigned char* in, const int* len, void* out, int B, int Tmax, int H, int W, int OH, int OW,
                    int dtype, int nhwc, xcp_stream_t stream);

/* ---- audio front end (XceptionLSTMA.py:44-46): F.interpolate(bilinear, align_corners=False) ----
 * out [NC][OH][OW] fp32 = bilinear resize of in [NC][IH][IW] fp32 (ATen's source-index and
 * weight formulas in fp32); MFCC frames [B*T*3][13][1] -> [B*T*3][64][64] */
int xcp_resize_bilinear(const float* in, float* out, int NC, int IH, int IW, int OH, int OW, xcp_stream_t stream);

/* ---- training step (train_visual.py:575-577): clip_grad_norm_ + Adam (L2 weight decay) ----
 * tab: DEVICE [nchunks][6] int64 (param, grad, exp_avg, exp_avg_sq, first element, length <= 16384),
 * all fp32.  xcp_opt_sumsq: out[0] = min(1, max_norm / (||g|| + 1e-6)) (1 if max_norm <= 0),
 * out[1] = ||g||, part = [nchunks] scratch.  xcp_opt_adam: g' = g * coef[0] (coef may be null),
 * g' += wd p; m = b1 m + (1-b1) g'; v = b2 v + (1-b2) g'^2; p -= lr / bc1 * m / (sqrt(v) / bc2sqrt + eps) */
int xcp_opt_sumsq(const long long* tab, int nchunks, float* part, float max_norm, float* out, xcp_stream_t stream);
int xcp_opt_adam(const long long* tab, int nchunks, const float* coef, float lr, float b1, float b2, float eps, float wd,
                 float bc1, float bc2sqrt, xcp_stream_t stream);
/* xcp_opt_adam with the step count t read from device memory (tdev[0]; the bias corrections formed on
 * the device in double from the double betas, as the host computes them): a graph-captured optimizer step */
int xcp_opt_adam_dev(const long long* tab, int nchunks, const float* coef, float lr, double b1, double b2, float eps,
                     float wd, const float* tdev, xcp_stream_t stream);

/* njobs permute3 jobs in one launch: jobs = DEVICE array [njobs][12] int64
 * (in, out, d0, d1, d2, p0, p1, p2, out dtype, first workgroup, s0, s1), nblocks workgroups in
 * total; output element (o0, o1, o2) goes to out[o0*s0 + o1*s1 + o2] (strides for the padded
 * layouts; dense: s1 = od2, s0 = od1*od2).  A job takes xcp_permute3_blocks(...) workgroups
 * (copies and 2-D transposes run as 32 x 32 tiles, other permutations one element per thread). */
int xcp_permute3_blocks(int d0, int d1, int d2, int p0, int p1, int p2, long s0, long s1);
int xcp_permute3_batch(const long long* jobs, int njobs, int nblocks, xcp_stream_t stream);

/* ---- classification heads / losses of the training scripts (fp32) ----
 * ArcFace (train_visual.py:455-474, m 0.5; train_au_face.py:423-442, m 0.30): X [B][D], W [C][D],
 * labels int64 [B] (null: plain s * cos), out [B][C] = s * cos(theta + m at the label, theta elsewhere);
 * xcp_arcface_bwd: dX [B][D], dW [C][D] from dout [B][C] (C <= 16).
 * Focal / class-weighted cross entropy (CBFocalLoss, train_au_face.py:445-458; gamma 0 and no
 * weights = nn.CrossEntropyLoss, train_visual.py:527): loss[0] = mean_i (1-pt_i)^gamma ce_i,
 * ce_i = w[y_i] (logsumexp(Z_i) - Z_i[y_i]), pt = exp(-ce); with dZ: dZ = gout[0] * dloss/dZ
 * (gout: device scalar, null = 1). */
int xcp_arcface_fwd(const float* X, const float* W, const long long* labels, float* out, int B, int C, int D, float s,
                    float m, xcp_stream_t stream);
int xcp_arcface_bwd(const float* X, const float* W, const long long* labels, const float* dout, float* dX, float* dW,
                    int B, int C, int D, float s, float m, xcp_stream_t stream);
int xcp_focal_ce(const float* Z, const long long* labels, const float* weights, float gamma, const float* gout,
                 float* loss, float* dZ, int B, int C, xcp_stream_t stream);

/* ---- LSTM recurrence (nn.LSTM, XceptionLSTMV.py:18-23, :67) ----
 * whh is W_hh [4H][H] as nn.LSTM stores it (weight_hh_l0); whhT ([H][4H]) is read only by the
 * generic kernel, i.e. when xcp_lstm_needs_whhT(B, H, kernel) returns 1 (H = 64 / 128 run
 * register-resident, H = 256 / 512 with B <= 32 on one persistent launch per direction -- W_hh
 * slices held in VGPRs by H / 4 workgroups that hand h_t / dgates_t over through L2 with sharded
 * step counters; H = 1024 (and 256 / 512 when the persistent grid cannot be resident, or with
 * XCP_LSTM_PERSIST=0) on per-step kernels while B fits their LDS budget).
 * kernel: 0 = automatic, 1 = the generic kernels.  xcp_lstm_bwd's work: max(B*H + 4*H*H, B*H*H/2)
 * floats (the per-step kernels' cell-gradient carry and a transposed W_hh; the persistent kernel's
 * double-buffered dh partials [2][B][H/4][H/4][4]). */
int xcp_lstm_needs_whhT(int B, int H, int kernel);
/* 1 if a persistent LSTM launch gave up waiting for its workgroups since the last call (its
 * outputs are then invalid; no wave spins forever), 0 if not, -1 on a HIP error.  Synchronises the
 * device and clears the flags. */
int xcp_lstm_sync_error(void);
int xcp_lstm_fwd(const float* xproj, const float* whh, const float* whhT, const float* bih, const float* bhh, float* out,
                 float* hprev, float* cst, float* gates, float* hn, float* cn, int B, int T, int H, int kernel,
                 xcp_stream_t stream);
int xcp_lstm_bwd(const float* dout, const float* dhn, const float* dcn, const float* whh, const float* cst,
                 const float* gates, float* dgates, float* work, int B, int T, int H, int kernel, xcp_stream_t stream);

/* ---- diagnostic (bench.py only; no reference counterpart) ----
 * blocks workgroups (one per CU) each run `iters` x 4 back-to-back bf16 MFMAs; out: DEVICE int64
 * [2 * blocks + 256]: out[2b] = shader cycles of block b's loop, out[2b + 1] = 100 MHz real-time
 * ticks of it (clock = cycles / ticks * 100 MHz). */
int xcp_clock_probe(long long* out, int blocks, int iters, xcp_stream_t stream);
/* out[i] = in[i] for n16 16-byte units (a multiple of 1024): the streaming-copy rate bench.py
 * quotes the depthwise kernels against (the guide's float4 copy) */
int xcp_stream_copy(const void* in, void* out, long n16, xcp_stream_t stream);
/* One-GPU stand-in for a bucket all-reduce (xcp.ddp proxy mode; no reference counterpart): `blocks`
 * workgroups copy n16 16-byte units in -> out and hold their CUs until `ticks` of the 100 MHz real-time
 * clock passed since each started.  rec: DEVICE uint64 [3], set to {UINT64_MAX, 0, 0} by the caller:
 * first workgroup start, last workgroup start, last workgroup end.  xcp_stamp: *out = max(*out, now) on
 * the same clock, as a stream marker. */
int xcp_comm_proxy(const void* in, void* out, long n16, int blocks, long long ticks, unsigned long long* rec,
                   xcp_stream_t stream);
int xcp_stamp(unsigned long long* out, xcp_stream_t stream);


#ifdef __cplusplus
}
#endif
#endif /* XCP_H_ */
