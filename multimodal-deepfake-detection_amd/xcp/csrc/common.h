// Shared device helpers for the xcp gfx950 kernels.
//
// Activations live in HBM as NHWC ("pixel rows of C channels"), dtype either
// fp32 (parity mode) or bf16 (throughput mode); accumulation is always fp32.
// Every kernel is templated on the storage type T through `Vec<T>` so the same
// source serves both modes.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define XCP_DEV __device__ __forceinline__

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned short u16x8 __attribute__((ext_vector_type(8)));
typedef unsigned short u16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

enum XcpDtype { XCP_F32 = 0, XCP_BF16 = 1 };

// error codes returned across the C-ABI (0 = success, otherwise hipError_t or these)
enum XcpStatus { XCP_OK = 0, XCP_EINVAL = 1001, XCP_EUNSUPPORTED = 1002 };
enum XcpFinFlags { XCP_FIN_ACCUMULATE = 1, XCP_FIN_NARROW = 2 };   // xcp_bn_bwd_finalize_part (include/xcp.h)

XCP_DEV float to_f(float x) { return x; }
XCP_DEV float to_f(bf16 x) { return (float)x; }
template <typename T> XCP_DEV T from_f(float x);
template <> XCP_DEV float from_f<float>(float x) { return x; }
template <> XCP_DEV bf16 from_f<bf16>(float x) { return (bf16)x; }

// round-trip through the storage type (used so BN statistics are taken over the
// values that are actually stored)
template <typename T> XCP_DEV float rnd(float x) { return to_f(from_f<T>(x)); }

// Load / store N consecutive elements as fp32.  N*sizeof(T) must be a multiple of
// 8 bytes and the address suitably aligned (channel counts are multiples of 8).
template <typename T, int N> struct VecIO;

template <int N> struct VecIO<float, N> {
  static XCP_DEV void load(const float* p, float* v) {
    if constexpr (N % 4 == 0) {
#pragma unroll
      for (int i = 0; i < N; i += 4) {
        float4 q = *reinterpret_cast<const float4*>(p + i);
        v[i] = q.x; v[i + 1] = q.y; v[i + 2] = q.z; v[i + 3] = q.w;
      }
    } else if constexpr (N == 1) {
      v[0] = *p;
    } else {
#pragma unroll
      for (int i = 0; i < N; i += 2) {
        float2 q = *reinterpret_cast<const float2*>(p + i);
        v[i] = q.x; v[i + 1] = q.y;
      }
    }
  }
  static XCP_DEV void store(float* p, const float* v) {
    if constexpr (N % 4 == 0) {
#pragma unroll
      for (int i = 0; i < N; i += 4)
        *reinterpret_cast<float4*>(p + i) = make_float4(v[i], v[i + 1], v[i + 2], v[i + 3]);
    } else if constexpr (N == 1) {
      *p = v[0];
    } else {
#pragma unroll
      for (int i = 0; i < N; i += 2) *reinterpret_cast<float2*>(p + i) = make_float2(v[i], v[i + 1]);
    }
  }
};

template <int N> struct VecIO<bf16, N> {
  static XCP_DEV void load(const bf16* p, float* v) {
    if constexpr (N % 8 == 0) {
#pragma unroll
      for (int i = 0; i < N; i += 8) {
        u16x8 q = *reinterpret_cast<const u16x8*>(p + i);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[i + j] = __uint_as_float(((unsigned)q[j]) << 16);
      }
    } else {
#pragma unroll
      for (int i = 0; i < N; i += 4) {
        u16x4 q = *reinterpret_cast<const u16x4*>(p + i);
#pragma unroll
        for (int j = 0; j < 4; ++j) v[i + j] = __uint_as_float(((unsigned)q[j]) << 16);
      }
    }
  }
  static XCP_DEV void store(bf16* p, const float* v) {
    if constexpr (N % 8 == 0) {
#pragma unroll
      for (int i = 0; i < N; i += 8) {
        bf16x8 q;
#pragma unroll
        for (int j = 0; j < 8; ++j) q[j] = (bf16)v[i + j];
        *reinterpret_cast<bf16x8*>(p + i) = q;
      }
    } else {
#pragma unroll
      for (int i = 0; i < N; i += 4) {
        bf16x4 q;
#pragma unroll
        for (int j = 0; j < 4; ++j) q[j] = (bf16)v[i + j];
        *reinterpret_cast<bf16x4*>(p + i) = q;
      }
    }
  }
};

XCP_DEV float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Input transform applied on load by consumers of a raw (pre-BN) tensor:
//   MODE_NONE: x;  MODE_RELU: max(x,0);  MODE_BNRELU: max(x*scale[c]+shift[c], 0)
enum XcpAct { ACT_NONE = 0, ACT_RELU = 1, ACT_BNRELU = 2 };

// Workgroup barrier that orders LDS only.  __syncthreads() also waits for every
// outstanding global store of the wave (vmcnt(0)); after an epilogue that has
// issued its stores that wait serialises the workgroup on store completion.
XCP_DEV void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// ds_read_b64_tr_b16: within each 16-lane group, lane 4q+p addresses row q, columns 4p..4p+3
// of a 4 x 16 bf16 block; lane i receives column i of the 4 rows
XCP_DEV bf16x4 ds_read_tr(const char* p) {
  typedef short s4 __attribute__((ext_vector_type(4)));
  s4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s4*)(p));
  return __builtin_bit_cast(bf16x4, v);
}

// two floats -> packed bf16 pair (a in the low half), one v_cvt_pk_bf16_f32 (round to nearest even, the
// same result as two scalar conversions; assigning the elements of a bf16 vector one at a time made
// hipcc convert each against a zero and merge the halves: 2-3 extra VALU per pair)
XCP_DEV unsigned pk_bf16(float a, float b) {
  return __builtin_bit_cast(unsigned, __builtin_convertvector(f32x2{a, b}, bf16x2));
}

static inline int xcp_cdiv(long a, long b) { return (int)((a + b - 1) / b); }

// Bijective XCD-aware remap of a linear workgroup id (cdna_hip_programming.md §5
// "XCD swizzle must be bijective"): blocks that share an XCD (id % 8) get a
// contiguous range of logical ids, so neighbouring tiles share that XCD's L2.
XCP_DEV int xcd_remap(int orig, int nwg) {
  const int q = nwg / 8, r = nwg % 8, xcd = orig % 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + orig / 8;
}
