// MFMA energy probe (gfx950): sustained bf16 MFMA issue with operands held in registers, on every
// CU, for a fixed wall time; prints the achieved TFLOP/s. scripts/mfma_power.py runs it under a
// board-power sampler to compare the FLOP per joule of v_mfma_f32_32x32x16_bf16 and
// v_mfma_f32_16x16x32_bf16 — on this power-capped chip (profiles/r3_power_step.log) the GEMM
// tile's MFMA shape is an energy choice, not only a throughput one: per FLOP the 32x32x16 form
// reads half the operand bytes from the register file.
//   build: hipcc --offload-arch=gfx950 -O3 csrc/tests/mfma_power_probe.hip -o build/mfma_power_probe
//   run:   build/mfma_power_probe <32|16|32z> <seconds>     (32z: zero operands)
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x16_t __attribute__((ext_vector_type(16)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));

// MFMAs as inline asm on "+a" accumulators (as csrc/kernels/gemm_w4.hip): the builtin's 16x16
// accumulators get shuffled through v_accvgpr_mov copies between iterations, halving the issue rate
__device__ __forceinline__ void m32(f32x16_t& c, const bf16x8_t& a, const bf16x8_t& b) {
  asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+a"(c) : "v"(a), "v"(b));
}
__device__ __forceinline__ void m16(f32x4_t& c, const bf16x8_t& a, const bf16x8_t& b) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(c) : "v"(a), "v"(b));
}

__device__ __forceinline__ bf16x8_t operand(unsigned seed, bool zero) {
  bf16x8_t r;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    unsigned x = seed * 2654435761u + i * 40503u;
    x ^= x >> 13;
    x *= 0x5bd1e995u;
    x ^= x >> 15;
    const float f = zero ? 0.f : ((float)(x & 0xffff) / 32768.f - 1.f);
    r[i] = (__bf16)f;
  }
  return r;
}

// 4 independent accumulator chains of 32x32x16 (32 K-FLOP each)
__global__ __launch_bounds__(256) void loop32(float* out, int iters, int zero) {
  const unsigned t = blockIdx.x * 256 + threadIdx.x;
  const bf16x8_t a = operand(t, zero), b = operand(t ^ 0x9e37u, zero);
  f32x16_t c0 = {}, c1 = {}, c2 = {}, c3 = {};
  for (int i = 0; i < iters; ++i) {
    m32(c0, a, b);
    m32(c1, b, a);
    m32(c2, a, a);
    m32(c3, b, b);
  }
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");  // MFMA results -> VALU reads
  float s = 0.f;
#pragma unroll
  for (int r = 0; r < 16; ++r) s += c0[r] + c1[r] + c2[r] + c3[r];
  out[t] = s;
}

// 8 independent accumulator chains of 16x16x32 (16 K-FLOP each): the same FLOPs per iteration
// (named accumulators: an array of them gets rotated through overlapping AGPR ranges)
__global__ __launch_bounds__(256) void loop16(float* out, int iters, int zero) {
  const unsigned t = blockIdx.x * 256 + threadIdx.x;
  const bf16x8_t a = operand(t, zero), b = operand(t ^ 0x9e37u, zero);
  f32x4_t c0 = {}, c1 = {}, c2 = {}, c3 = {}, c4 = {}, c5 = {}, c6 = {}, c7 = {};
  for (int i = 0; i < iters; ++i) {
    m16(c0, a, b);
    m16(c1, b, a);
    m16(c2, a, a);
    m16(c3, b, b);
    m16(c4, a, b);
    m16(c5, b, a);
    m16(c6, a, a);
    m16(c7, b, b);
  }
  asm volatile("s_nop 7\n\ts_nop 7" ::: "memory");
  const f32x4_t s4 = c0 + c1 + c2 + c3 + c4 + c5 + c6 + c7;
  out[t] = s4[0] + s4[1] + s4[2] + s4[3];
}

int main(int argc, char** argv) {
  const char* mode = argc > 1 ? argv[1] : "32";
  const double secs = argc > 2 ? atof(argv[2]) : 3.0;
  const bool is32 = mode[0] == '3', zero = strchr(mode, 'z') != nullptr;
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  const int blocks = cus * 2;  // 2 waves per SIMD
  float* out;
  if (hipMalloc(&out, (size_t)blocks * 256 * sizeof(float)) != hipSuccess) return 1;
  const int iters = 4096;
  const double flop_per_launch = (double)blocks * 4 /*waves*/ * iters * 4 * 32768.0;  // both kernels
  auto launch = [&] {
    if (is32)
      hipLaunchKernelGGL(loop32, dim3(blocks), dim3(256), 0, 0, out, iters, (int)zero);
    else
      hipLaunchKernelGGL(loop16, dim3(blocks), dim3(256), 0, 0, out, iters, (int)zero);
  };
  launch();
  hipDeviceSynchronize();
  const auto t0 = std::chrono::steady_clock::now();
  long n = 0;
  double el = 0;
  while (el < secs) {
    for (int k = 0; k < 8; ++k) launch();
    hipDeviceSynchronize();
    n += 8;
    el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  }
  printf("mode %s: %ld launches in %.2f s: %.0f TFLOP/s\n", mode, n, el, n * flop_per_launch / el / 1e12);
  hipFree(out);
  return 0;
}
