// Host-side glue between at::Tensor and the gfx950 kernels.
#pragma once

#include <cstdlib>

#include <ATen/ATen.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>
#include <c10/core/DeviceGuard.h>
#include <torch/library.h>

#include "common.h"

// FT_EXACT_MATH=1: IEEE-exact division / sqrt in the element-wise update kernels (AdamW, SwiGLU)
// instead of the hardware v_rcp_f32 / v_sqrt_f32 (common.h fast_rcp); same-process A/B through
// torch.ops.ftamd.set_exact_math.
inline bool& ft_exact_math() {
  static bool v = [] {
    const char* e = std::getenv("FT_EXACT_MATH");
    return e != nullptr && std::atoi(e) != 0;
  }();
  return v;
}

static inline hipStream_t ft_stream() {
  return at::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream();
}

#define FT_CHECK_CUDA(t) TORCH_CHECK((t).is_cuda(), #t " must be a GPU tensor")
#define FT_CHECK_CONTIG(t) TORCH_CHECK((t).is_contiguous(), #t " must be contiguous")
#define FT_CHECK_BF16(t) TORCH_CHECK((t).scalar_type() == at::kBFloat16, #t " must be bf16")
#define FT_CHECK_F32(t) TORCH_CHECK((t).scalar_type() == at::kFloat, #t " must be fp32")

#define FT_LAUNCH_CHECK() FT_HIP_CHECK(hipGetLastError())

// model dtypes with hand-written kernels: bf16 (default), fp16, fp32
#define FT_CHECK_MODEL_DTYPE(t)                                                                           \
  TORCH_CHECK((t).scalar_type() == at::kBFloat16 || (t).scalar_type() == at::kHalf ||                   \
                  (t).scalar_type() == at::kFloat,                                                      \
              #t " must be bf16, fp16 or fp32")

// Runs BODY with E = the element type of scalar type ST (EBF16 / EF16 / EF32).
#define FT_DISPATCH_E(ST, ...)                   \
  do {                                           \
    const auto _st = (ST);                       \
    if (_st == at::kBFloat16) {                  \
      using E = EBF16;                           \
      __VA_ARGS__;                               \
    } else if (_st == at::kHalf) {               \
      using E = EF16;                            \
      __VA_ARGS__;                               \
    } else if (_st == at::kFloat) {              \
      using E = EF32;                            \
      __VA_ARGS__;                               \
    } else {                                     \
      TORCH_CHECK(false, "unsupported dtype ", _st); \
    }                                            \
  } while (0)

// Same for the 16-bit model dtypes only (MFMA kernels: bf16 / fp16).
#define FT_DISPATCH_E16(ST, ...)                 \
  do {                                           \
    const auto _st = (ST);                       \
    if (_st == at::kBFloat16) {                  \
      using E = EBF16;                           \
      __VA_ARGS__;                               \
    } else if (_st == at::kHalf) {               \
      using E = EF16;                            \
      __VA_ARGS__;                               \
    } else {                                     \
      TORCH_CHECK(false, "unsupported dtype ", _st, " (bf16 / fp16 only)"); \
    }                                            \
  } while (0)

template <typename T>
static inline const T* cptr(const at::Tensor& t) {
  return reinterpret_cast<const T*>(t.data_ptr());
}
template <typename T>
static inline T* mptr(const at::Tensor& t) {
  return reinterpret_cast<T*>(t.data_ptr());
}
