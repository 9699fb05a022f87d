// Shared helpers for the gfx950 (CDNA4) kernels.
//
// All kernels are written for wave64 and 16-byte vector memory access
// (cdna_hip_programming.md Guideline 13). bf16 is carried as raw uint16 bits
// and converted with the native __bf16 type, which hipcc lowers to
// v_cvt_pk_bf16_f32 on gfx950 (round-to-nearest-even, NaN preserving).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#define FT_WAVE 64

typedef uint16_t bf16_t;
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4_t __attribute__((ext_vector_type(4)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));
typedef float f32x16_t __attribute__((ext_vector_type(16)));

// Hardware reciprocal / square root (v_rcp_f32 / v_sqrt_f32, 1 ulp): the IEEE-exact `1.f / x`
// and `sqrtf` expand to ~10 instructions each (v_div_scale x2, v_div_fmas, v_div_fixup, Newton
// steps; denormal scaling around v_sqrt), which made the element-wise update kernels issue-heavy
// (AdamW: 54 instructions per element). Their results are rounded to bf16 / fp16 (8 / 11-bit
// mantissas) or kept as fp32 moments where a 1-ulp difference is far below the update's own noise.
// On this power-capped chip (profiles/r3_power_step.log) every instruction a streaming kernel
// does not issue is power the concurrent GEMMs can spend.
__device__ __forceinline__ float fast_rcp(float x) { return __builtin_amdgcn_rcpf(x); }
__device__ __forceinline__ float fast_sqrt(float x) { return __builtin_amdgcn_sqrtf(x); }
// logistic sigmoid; `exact` (uniform): IEEE division instead of v_rcp_f32 (FT_EXACT_MATH A/B)
__device__ __forceinline__ float sigmoid_f(float x, bool exact) {
  const float d = 1.f + __expf(-x);
  return exact ? 1.f / d : fast_rcp(d);
}

// d/dg, d/du of silu(g) * u given the upstream d, with every fma explicit so the element-wise
// kernels (swiglu.hip) and the GEMM epilogue (gemm_w4.hip) round identically (the contraction the
// compiler picks otherwise differs by kernel once the division is a plain v_rcp_f32).
__device__ __forceinline__ void swiglu_grad(float g, float u, float d, bool exact, float& dg, float& du) {
  const float s = sigmoid_f(g, exact);
  const float silu = g * s;
  du = d * silu;
  dg = (d * u) * fmaf(silu, 1.f - s, s);
}

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

// ---- element types of the model dtype (--model-dtype bf16 / fp16 / fp32, reference utils.py:14-19):
// storage T, math in fp32. 8 elements move per access: 16 B for the 16-bit types, 32 B for fp32.
struct EBF16 {
  typedef uint16_t T;
  static constexpr bool is16 = true;
};
struct EF16 {
  typedef uint16_t T;
  static constexpr bool is16 = true;
};
struct EF32 {
  typedef float T;
  static constexpr bool is16 = false;
};

__device__ __forceinline__ float h2f(uint16_t v) { return (float)__builtin_bit_cast(_Float16, v); }
__device__ __forceinline__ uint16_t f2h(float f) { return __builtin_bit_cast(uint16_t, (_Float16)f); }

template <class E>
__device__ __forceinline__ float ld1(const typename E::T* p) {
  if constexpr (std::is_same<E, EBF16>::value) return bf2f(*p);
  else if constexpr (std::is_same<E, EF16>::value) return h2f(*p);
  else return *p;
}

template <class E>
__device__ __forceinline__ typename E::T cvt1(float f) {
  if constexpr (std::is_same<E, EBF16>::value) return f2bf(f);
  else if constexpr (std::is_same<E, EF16>::value) return f2h(f);
  else return f;
}

// 8 elements kept packed in registers (one uint4 for the 16-bit types, two for fp32):
// kernels that hold whole rows between passes keep them packed and unpack per pass.
template <class E>
struct P8 {
  uint4 v[E::is16 ? 1 : 2];
};

template <class E>
__device__ __forceinline__ P8<E> ldp8(const typename E::T* p) {
  P8<E> r;
  r.v[0] = *reinterpret_cast<const uint4*>(p);
  if constexpr (!E::is16) r.v[1] = *reinterpret_cast<const uint4*>(p + 4);
  return r;
}

template <class E>
__device__ __forceinline__ P8<E> zp8() {
  P8<E> r;
#pragma unroll
  for (int i = 0; i < (E::is16 ? 1 : 2); ++i) r.v[i] = make_uint4(0, 0, 0, 0);
  return r;
}

// Opaque register barrier: keeps the packed values (not their fp32 unpack) live.
template <class E>
__device__ __forceinline__ void pin8(P8<E>& r) {
#pragma unroll
  for (int i = 0; i < (E::is16 ? 1 : 2); ++i)
    asm volatile("" : "+v"(r.v[i].x), "+v"(r.v[i].y), "+v"(r.v[i].z), "+v"(r.v[i].w));
}

template <class E>
__device__ __forceinline__ void unp8(const P8<E>& r, float* f) {
  if constexpr (std::is_same<E, EBF16>::value) {
    unpack8(r.v[0], f);
  } else if constexpr (std::is_same<E, EF16>::value) {
    const uint32_t w[4] = {r.v[0].x, r.v[0].y, r.v[0].z, r.v[0].w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      f[2 * i] = h2f((uint16_t)(w[i] & 0xffffu));
      f[2 * i + 1] = h2f((uint16_t)(w[i] >> 16));
    }
  } else {
    f[0] = __uint_as_float(r.v[0].x); f[1] = __uint_as_float(r.v[0].y);
    f[2] = __uint_as_float(r.v[0].z); f[3] = __uint_as_float(r.v[0].w);
    f[4] = __uint_as_float(r.v[1].x); f[5] = __uint_as_float(r.v[1].y);
    f[6] = __uint_as_float(r.v[1].z); f[7] = __uint_as_float(r.v[1].w);
  }
}

// Round through the model dtype (identity for fp32).
template <class E>
__device__ __forceinline__ float rnd(float f) {
  if constexpr (std::is_same<E, EF32>::value) return f;
  else {
    const typename E::T t = cvt1<E>(f);
    return ld1<E>(&t);
  }
}

template <class E>
__device__ __forceinline__ void ld8(const typename E::T* p, float* f) {
  unp8<E>(ldp8<E>(p), f);
}

template <class E>
__device__ __forceinline__ P8<E> pk8(const float* f) {
  P8<E> r;
  if constexpr (std::is_same<E, EBF16>::value) {
    r.v[0] = pack8(f);
  } else if constexpr (std::is_same<E, EF16>::value) {
    r.v[0].x = (uint32_t)f2h(f[0]) | ((uint32_t)f2h(f[1]) << 16);
    r.v[0].y = (uint32_t)f2h(f[2]) | ((uint32_t)f2h(f[3]) << 16);
    r.v[0].z = (uint32_t)f2h(f[4]) | ((uint32_t)f2h(f[5]) << 16);
    r.v[0].w = (uint32_t)f2h(f[6]) | ((uint32_t)f2h(f[7]) << 16);
  } else {
    r.v[0] = make_uint4(__float_as_uint(f[0]), __float_as_uint(f[1]), __float_as_uint(f[2]),
                        __float_as_uint(f[3]));
    r.v[1] = make_uint4(__float_as_uint(f[4]), __float_as_uint(f[5]), __float_as_uint(f[6]),
                        __float_as_uint(f[7]));
  }
  return r;
}

template <class E>
__device__ __forceinline__ void st8(typename E::T* p, const float* f) {
  const P8<E> r = pk8<E>(f);
  *reinterpret_cast<uint4*>(p) = r.v[0];
  if constexpr (!E::is16) *reinterpret_cast<uint4*>(p + 4) = r.v[1];
}

// 16-bit element types: 8 values in one uint4 <-> 8 floats; 2 floats -> one packed pair.
template <class E>
__device__ __forceinline__ void unpack8e(const uint4& v, float* f) {
  static_assert(E::is16, "16-bit element types only");
  P8<E> r;
  r.v[0] = v;
  unp8<E>(r, f);
}
template <class E>
__device__ __forceinline__ uint4 pack8e(const float* f) {
  static_assert(E::is16, "16-bit element types only");
  return pk8<E>(f).v[0];
}
template <class E>
__device__ __forceinline__ uint32_t pk2(float lo, float hi) {
  static_assert(E::is16, "16-bit element types only");
  return (uint32_t)cvt1<E>(lo) | ((uint32_t)cvt1<E>(hi) << 16);
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
