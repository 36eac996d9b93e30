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

}  // namespace

extern "C" {

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

}  // extern "C"
