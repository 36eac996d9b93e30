// Clip input conversion on the GPU: uint8 face frames -> the model's fp32 input.
//
// Reference: FaceDataset.__getitem__ (video_dataloader.py:22-37) turns an .npy clip of
// uint8 [T, H, W, 3] into fp32 [T, 3, H, W] / 255 (no mean / std), and collate_fn
// (video_dataloader.py:53-68) zero-pads T to the batch maximum.  Done on the host that is
// 4 bytes per subpixel over PCIe; here the host ships the uint8 clips (a quarter of the
// bytes) and this kernel expands them in HBM, bit-identical to the host path (the same
// IEEE single-precision x / 255).
//
// in  [B][Tmax][H][W][3] uint8 (frames t >= len[b] are ignored, their output is zero)
// out [B][Tmax][3][H][W] fp32
// One thread converts 4 consecutive pixels of one row: one 12-byte read, three 16-byte
// stores (one per channel plane).  HBM-bound: 3 + 12 bytes per pixel.
#include "common.h"

namespace {

__global__ __launch_bounds__(256) void frames_u8_kernel(const unsigned char* __restrict__ in,
                                                        const int* __restrict__ len, float* __restrict__ out, int Tmax,
                                                        int H, int W, long total) {
  const int W4 = W / 4;
  const long g = (long)blockIdx.x * 256 + threadIdx.x;
  if (g >= total) return;
  const long per_frame = (long)H * W4;
  const long frame = g / per_frame;               // b * Tmax + t
  const long r = g - frame * per_frame;
  const int h = (int)(r / W4), w0 = (int)(r - (long)h * W4) * 4;
  const int b = (int)(frame / Tmax), t = (int)(frame - (long)b * Tmax);
  float v[3][4];
  if (t < len[b]) {
    const unsigned* src = reinterpret_cast<const unsigned*>(in + ((frame * H + h) * W + w0) * 3);
    const unsigned u[3] = {src[0], src[1], src[2]};   // 12 bytes: pixels w0..w0+3, RGB interleaved
#pragma unroll
    for (int k = 0; k < 12; ++k) {
      const unsigned byte = (u[k >> 2] >> (8 * (k & 3))) & 0xffu;
      v[k % 3][k / 3] = (float)byte / 255.f;
    }
  } else {
#pragma unroll
    for (int c = 0; c < 3; ++c)
#pragma unroll
      for (int p = 0; p < 4; ++p) v[c][p] = 0.f;
  }
#pragma unroll
  for (int c = 0; c < 3; ++c)
    *reinterpret_cast<float4*>(out + (((frame * 3 + c) * H + h) * W + w0)) = make_float4(v[c][0], v[c][1], v[c][2], v[c][3]);
}


// Bilinear resize, align_corners=False (F.interpolate(..., mode="bilinear"), as the audio
// front end XceptionLSTMA.py:46 uses it: MFCC [B*T, 3, 13, 1] -> [B*T, 3, 64, 64]).
// Source coordinates, indices and weights follow ATen's upsample_bilinear2d in fp32:
//   src = max(scale * (dst + 0.5) - 0.5, 0), scale = in / out, i0 = min(floor(src), in - 1),
//   i1 = i0 + (i0 < in - 1), l1 = clamp(src - i0, 0, 1), l0 = 1 - l1,
//   out = (a * w0 + b * w1) * h0 + (c * w0 + d * w1) * h1  (products, then sums).
// in [NC][IH][IW], out [NC][OH][OW] fp32; one thread per output pixel.
XCP_DEV void lin_idx(int dst, int in, float scale, int& i0, int& i1, float& l0, float& l1) {
#pragma clang fp contract(off)
  float src = scale * ((float)dst + 0.5f) - 0.5f;
  src = src < 0.f ? 0.f : src;
  i0 = min((int)floorf(src), in - 1);
  i1 = i0 + (i0 < in - 1 ? 1 : 0);
  float l = src - (float)i0;
  l = l < 0.f ? 0.f : (l > 1.f ? 1.f : l);
  l1 = l;
  l0 = 1.f - l;
}

__global__ __launch_bounds__(256) void resize_bilinear_kernel(const float* __restrict__ in, float* __restrict__ out,
                                                              int IH, int IW, int OH, int OW, float sh, float sw,
                                                              long total) {
#pragma clang fp contract(off)
  const long g = (long)blockIdx.x * 256 + threadIdx.x;
  if (g >= total) return;
  const long plane = g / ((long)OH * OW);
  const int r = (int)(g - plane * OH * OW), oh = r / OW, ow = r - oh * OW;
  int h0, h1, w0, w1;
  float lh0, lh1, lw0, lw1;
  lin_idx(oh, IH, sh, h0, h1, lh0, lh1);
  lin_idx(ow, IW, sw, w0, w1, lw0, lw1);
  const float* p = in + plane * IH * IW;
  const float t0 = p[h0 * IW + w0] * lw0 + p[h0 * IW + w1] * lw1;
  const float t1 = p[h1 * IW + w0] * lw0 + p[h1 * IW + w1] * lw1;
  out[g] = t0 * lh0 + t1 * lh1;
}

// General clip preparation: uint8 frames -> x / 255, optionally bilinear-resized to OH x OW
// (F.interpolate(x / 255, (OH, OW), mode="bilinear", align_corners=False) of the fp32 clip, as
// lin_idx above), stored fp32 or bf16 (round to nearest even of that fp32 value), planar
// [B][Tmax][3][OH][OW] or interleaved [B][Tmax][OH][OW][3].  One thread per output pixel
// (3 channels); frames past a clip's length are zero.
template <typename T, bool NHWC>
__global__ __launch_bounds__(256) void frames_prep_kernel(const unsigned char* __restrict__ in,
                                                          const int* __restrict__ len, T* __restrict__ out, int Tmax,
                                                          int H, int W, int OH, int OW, float sh, float sw, long total) {
#pragma clang fp contract(off)
  const long g = (long)blockIdx.x * 256 + threadIdx.x;
  if (g >= total) return;
  const long per_frame = (long)OH * OW;
  const long frame = g / per_frame;
  const int r = (int)(g - frame * per_frame), oh = r / OW, ow = r - oh * OW;
  const int b = (int)(frame / Tmax), t = (int)(frame - (long)b * Tmax);
  float v[3] = {0.f, 0.f, 0.f};
  if (t < len[b]) {
    const unsigned char* f = in + frame * H * W * 3;
    if (OH == H && OW == W) {
#pragma unroll
      for (int c = 0; c < 3; ++c) v[c] = (float)f[((long)oh * W + ow) * 3 + c] / 255.f;
    } else {
      int h0, h1, w0, w1;
      float lh0, lh1, lw0, lw1;
      lin_idx(oh, H, sh, h0, h1, lh0, lh1);
      lin_idx(ow, W, sw, w0, w1, lw0, lw1);
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        const float a = (float)f[((long)h0 * W + w0) * 3 + c] / 255.f, bb = (float)f[((long)h0 * W + w1) * 3 + c] / 255.f;
        const float cc = (float)f[((long)h1 * W + w0) * 3 + c] / 255.f, d = (float)f[((long)h1 * W + w1) * 3 + c] / 255.f;
        const float t0 = a * lw0 + bb * lw1;
        const float t1 = cc * lw0 + d * lw1;
        v[c] = t0 * lh0 + t1 * lh1;
      }
    }
  }
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const long o = NHWC ? g * 3 + c : ((frame * 3 + c) * OH + oh) * OW + ow;
    out[o] = (T)v[c];
  }
}

template <typename T>
void launch_prep(const unsigned char* in, const int* len, void* out, bool nhwc, int Tmax, int H, int W, int OH, int OW,
                 long total, hipStream_t st) {
  const dim3 grid((unsigned)((total + 255) / 256));
  const float sh = (float)H / (float)OH, sw = (float)W / (float)OW;
  if (nhwc)
    hipLaunchKernelGGL((frames_prep_kernel<T, true>), grid, dim3(256), 0, st, in, len, (T*)out, Tmax, H, W, OH, OW, sh,
                       sw, total);
  else
    hipLaunchKernelGGL((frames_prep_kernel<T, false>), grid, dim3(256), 0, st, in, len, (T*)out, Tmax, H, W, OH, OW, sh,
                       sw, total);
}

}  // namespace

extern "C" {

// B clips of up to Tmax uint8 [H][W][3] frames (len: device int32 [B]) -> out at OH x OW:
// dtype XCP_F32 / XCP_BF16, nhwc 0 = [B][Tmax][3][OH][OW], 1 = [B][Tmax][OH][OW][3]
int xcp_frames_prep(const unsigned char* in, const int* len, void* out, int B, int Tmax, int H, int W, int OH, int OW,
                    int dtype, int nhwc, hipStream_t st) {
  if (B <= 0 || Tmax <= 0 || OH <= 0 || OW <= 0) return XCP_OK;
  if (H <= 0 || W <= 0 || (dtype != XCP_F32 && dtype != XCP_BF16)) return XCP_EINVAL;
  const long total = (long)B * Tmax * OH * OW;
  if (dtype == XCP_F32)
    launch_prep<float>(in, len, out, nhwc != 0, Tmax, H, W, OH, OW, total, st);
  else
    launch_prep<bf16>(in, len, out, nhwc != 0, Tmax, H, W, OH, OW, total, st);
  return (int)hipGetLastError();
}

// B clips of up to Tmax frames (len: device int32 [B]); W must be a multiple of 4
int xcp_frames_u8_to_f32(const unsigned char* in, const int* len, float* out, int B, int Tmax, int H, int W,
                         hipStream_t st) {
  if (B <= 0 || Tmax <= 0 || H <= 0 || W <= 0) return XCP_OK;
  if (W % 4) return XCP_EINVAL;
  const long total = (long)B * Tmax * H * (W / 4);
  hipLaunchKernelGGL(frames_u8_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, in, len, out, Tmax, H,
                     W, total);
  return (int)hipGetLastError();
}

// out [NC][OH][OW] = bilinear resize (align_corners=False) of in [NC][IH][IW], fp32
int xcp_resize_bilinear(const float* in, float* out, int NC, int IH, int IW, int OH, int OW, hipStream_t st) {
  if (NC <= 0 || OH <= 0 || OW <= 0) return XCP_OK;
  if (IH <= 0 || IW <= 0) return XCP_EINVAL;
  const long total = (long)NC * OH * OW;
  hipLaunchKernelGGL(resize_bilinear_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, in, out, IH, IW,
                     OH, OW, (float)IH / (float)OH, (float)IW / (float)OW, total);
  return (int)hipGetLastError();
}

}  // extern "C"
