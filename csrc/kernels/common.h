// Shared helpers for the gfx950 (CDNA4) kernels.
//
// All kernels are written for wave64 and 16-byte vector memory access
// (cdna_hip_programming.md Guideline 13). bf16 is carried as raw uint16 bits
// and converted with the native __bf16 type, which hipcc lowers to
// v_cvt_pk_bf16_f32 on gfx950 (round-to-nearest-even, NaN preserving).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#define FT_WAVE 64

typedef uint16_t bf16_t;
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4_t __attribute__((ext_vector_type(4)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));
typedef float f32x16_t __attribute__((ext_vector_type(16)));

__device__ __forceinline__ float bf2f(bf16_t v) { return __uint_as_float(((uint32_t)v) << 16); }

__device__ __forceinline__ bf16_t f2bf(float f) {
  __bf16 b = (__bf16)f;
  return __builtin_bit_cast(bf16_t, b);
}

// 8 x bf16 packed in a uint4 <-> 8 floats.
__device__ __forceinline__ void unpack8(const uint4& v, float* f) {
  f[0] = __uint_as_float(v.x << 16);
  f[1] = __uint_as_float(v.x & 0xffff0000u);
  f[2] = __uint_as_float(v.y << 16);
  f[3] = __uint_as_float(v.y & 0xffff0000u);
  f[4] = __uint_as_float(v.z << 16);
  f[5] = __uint_as_float(v.z & 0xffff0000u);
  f[6] = __uint_as_float(v.w << 16);
  f[7] = __uint_as_float(v.w & 0xffff0000u);
}

__device__ __forceinline__ uint32_t pack2(float lo, float hi) {
  return (uint32_t)f2bf(lo) | ((uint32_t)f2bf(hi) << 16);
}

__device__ __forceinline__ uint4 pack8(const float* f) {
  uint4 r;
  r.x = pack2(f[0], f[1]);
  r.y = pack2(f[2], f[3]);
  r.z = pack2(f[4], f[5]);
  r.w = pack2(f[6], f[7]);
  return r;
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Block-wide sum for blockDim.x == NT (multiple of 64). `red` needs NT/64 floats.
template <int NT>
__device__ __forceinline__ float block_sum(float v, float* red) {
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) red[wid] = v;
  __syncthreads();
  float t = 0.f;
#pragma unroll
  for (int i = 0; i < NT / 64; ++i) t += red[i];
  __syncthreads();
  return t;
}

#define FT_HIP_CHECK(expr)                                                              \
  do {                                                                                 \
    hipError_t _e = (expr);                                                            \
    TORCH_CHECK(_e == hipSuccess, "HIP error ", hipGetErrorString(_e), " at ", __FILE__, \
                ":", __LINE__);                                                        \
  } while (0)
