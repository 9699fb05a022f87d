// SwiGLU activation on the fused up/gate projection, forward + backward.
//
// Parity: reference model.py:253-254 `w2(silu(w1 x) * w3 x)`. The two input
// projections run as ONE GEMM against the concatenated [w1; w3] weight (they
// are adjacent in the flat parameter buffer), so this kernel reads gu =
// [T, 2F] (gate in columns [0,F), up in [F,2F)) and writes a = silu(g) * u.
// fp32 math, one rounding per output (the reference rounds twice). bf16 / fp16 / fp32
// (--model-dtype); 16-B (32-B for fp32) vector accesses, grid-stride. (On the Llama-3-8B path
// both directions run inside the w4 GEMM epilogues instead: gemm_w4.h W4_SWIGLU / W4_SWIGLU_BWD.)
#include "torch_utils.h"

namespace {


template <class E>
__global__ __launch_bounds__(256) void swiglu_fwd_kernel(const typename E::T* __restrict__ gu,
                                                         typename E::T* __restrict__ a, long T, int F, int exact) {
  const int vpr = F >> 3;
  const long total = T * vpr;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total;
       i += (long)gridDim.x * blockDim.x) {
    const long row = i / vpr;
    const int col = (int)(i - row * vpr) * 8;
    float g[8], u[8], o[8];
    ld8<E>(gu + row * 2 * F + col, g);
    ld8<E>(gu + row * 2 * F + F + col, u);
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = g[j] * sigmoid_f(g[j], exact) * u[j];
    st8<E>(a + row * F + col, o);
  }
}

template <class E>
__global__ __launch_bounds__(256) void swiglu_bwd_kernel(const typename E::T* __restrict__ da,
                                                         const typename E::T* __restrict__ gu,
                                                         typename E::T* __restrict__ dgu, long T, int F, int exact) {
  const int vpr = F >> 3;
  const long total = T * vpr;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total;
       i += (long)gridDim.x * blockDim.x) {
    const long row = i / vpr;
    const int col = (int)(i - row * vpr) * 8;
    float g[8], u[8], d[8], dg[8], du[8];
    ld8<E>(gu + row * 2 * F + col, g);
    ld8<E>(gu + row * 2 * F + F + col, u);
    ld8<E>(da + row * F + col, d);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      swiglu_grad(g[j], u[j], d[j], exact, dg[j], du[j]);
    }
    st8<E>(dgu + row * 2 * F + col, dg);
    st8<E>(dgu + row * 2 * F + F + col, du);
  }
}

int grid_for(long work) {
  long g = (work + 255) / 256;
  return (int)std::max(1L, std::min(g, 256L * 16));
}

}  // namespace

at::Tensor swiglu_fwd(const at::Tensor& gu) {
  FT_CHECK_CUDA(gu);
  FT_CHECK_MODEL_DTYPE(gu);
  FT_CHECK_CONTIG(gu);
  const int F2 = gu.size(-1);
  TORCH_CHECK(F2 % 16 == 0, "swiglu: 2F must be a multiple of 16");
  const int F = F2 / 2;
  const long T = gu.numel() / F2;
  const at::DeviceGuard guard(gu.device());
  auto sizes = gu.sizes().vec();
  sizes.back() = F;
  auto a = at::empty(sizes, gu.options());
  const long work = T * (F / 8);
  if (work > 0)
    FT_DISPATCH_E(gu.scalar_type(),
                  hipLaunchKernelGGL(swiglu_fwd_kernel<E>, dim3(grid_for(work)), dim3(256), 0, ft_stream(),
                                     cptr<typename E::T>(gu), mptr<typename E::T>(a), T, F, (int)ft_exact_math()));
  FT_LAUNCH_CHECK();
  return a;
}

at::Tensor swiglu_bwd(const at::Tensor& da, const at::Tensor& gu) {
  FT_CHECK_CUDA(da);
  FT_CHECK_MODEL_DTYPE(da);
  TORCH_CHECK(da.scalar_type() == gu.scalar_type(), "swiglu_bwd: dtype mismatch");
  FT_CHECK_CONTIG(da);
  FT_CHECK_CONTIG(gu);
  const int F2 = gu.size(-1);
  const int F = F2 / 2;
  const long T = gu.numel() / F2;
  TORCH_CHECK(da.numel() == T * F, "swiglu_bwd: shape mismatch");
  const at::DeviceGuard guard(gu.device());
  auto dgu = at::empty_like(gu);
  const long work = T * (F / 8);
  if (work > 0)
    FT_DISPATCH_E(gu.scalar_type(),
                  hipLaunchKernelGGL(swiglu_bwd_kernel<E>, dim3(grid_for(work)), dim3(256), 0, ft_stream(),
                                     cptr<typename E::T>(da), cptr<typename E::T>(gu), mptr<typename E::T>(dgu),
                                     T, F, (int)ft_exact_math()));
  FT_LAUNCH_CHECK();
  return dgu;
}

// Same-process A/B of the IEEE-exact vs hardware reciprocal / sqrt (see ft_exact_math).
void set_exact_math(bool on) { ft_exact_math() = on; }

TORCH_LIBRARY_FRAGMENT(ftamd, m) {
  m.def("set_exact_math(bool on) -> ()", &set_exact_math);
  m.def("swiglu_fwd(Tensor gu) -> Tensor", &swiglu_fwd);
  m.def("swiglu_bwd(Tensor da, Tensor gu) -> Tensor", &swiglu_bwd);
}
