// SwiGLU activation on the fused up/gate projection, forward + backward.
//
// Parity: reference model.py:253-254 `w2(silu(w1 x) * w3 x)`. The two input
// projections run as ONE GEMM against the concatenated [w1; w3] weight (they
// are adjacent in the flat parameter buffer), so this kernel reads gu =
// [T, 2F] (gate in columns [0,F), up in [F,2F)) and writes a = silu(g) * u.
// fp32 math, one bf16 rounding per output (the reference rounds twice).
// 16-B vector accesses, grid-stride.
#include "torch_utils.h"

namespace {

__device__ __forceinline__ float sigmoidf_(float x) { return 1.f / (1.f + __expf(-x)); }

__global__ __launch_bounds__(256) void swiglu_fwd_kernel(const bf16_t* __restrict__ gu,
                                                         bf16_t* __restrict__ a, long T, int F) {
  const int vpr = F >> 3;
  const long total = T * vpr;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total;
       i += (long)gridDim.x * blockDim.x) {
    const long row = i / vpr;
    const int col = (int)(i - row * vpr) * 8;
    float g[8], u[8], o[8];
    unpack8(*reinterpret_cast<const uint4*>(gu + row * 2 * F + col), g);
    unpack8(*reinterpret_cast<const uint4*>(gu + row * 2 * F + F + col), u);
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = g[j] * sigmoidf_(g[j]) * u[j];
    *reinterpret_cast<uint4*>(a + row * F + col) = pack8(o);
  }
}

__global__ __launch_bounds__(256) void swiglu_bwd_kernel(const bf16_t* __restrict__ da,
                                                         const bf16_t* __restrict__ gu,
                                                         bf16_t* __restrict__ dgu, long T, int F) {
  const int vpr = F >> 3;
  const long total = T * vpr;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total;
       i += (long)gridDim.x * blockDim.x) {
    const long row = i / vpr;
    const int col = (int)(i - row * vpr) * 8;
    float g[8], u[8], d[8], dg[8], du[8];
    unpack8(*reinterpret_cast<const uint4*>(gu + row * 2 * F + col), g);
    unpack8(*reinterpret_cast<const uint4*>(gu + row * 2 * F + F + col), u);
    unpack8(*reinterpret_cast<const uint4*>(da + row * F + col), d);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float s = sigmoidf_(g[j]);
      const float silu = g[j] * s;
      du[j] = d[j] * silu;
      dg[j] = d[j] * u[j] * (s + silu * (1.f - s));
    }
    *reinterpret_cast<uint4*>(dgu + row * 2 * F + col) = pack8(dg);
    *reinterpret_cast<uint4*>(dgu + row * 2 * F + F + col) = pack8(du);
  }
}

int grid_for(long work) {
  long g = (work + 255) / 256;
  return (int)std::max(1L, std::min(g, 256L * 16));
}

}  // namespace

at::Tensor swiglu_fwd(const at::Tensor& gu) {
  FT_CHECK_CUDA(gu);
  FT_CHECK_BF16(gu);
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
    hipLaunchKernelGGL(swiglu_fwd_kernel, dim3(grid_for(work)), dim3(256), 0, ft_stream(),
                       cptr<bf16_t>(gu), mptr<bf16_t>(a), T, F);
  FT_LAUNCH_CHECK();
  return a;
}

at::Tensor swiglu_bwd(const at::Tensor& da, const at::Tensor& gu) {
  FT_CHECK_CUDA(da);
  FT_CHECK_BF16(da);
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
    hipLaunchKernelGGL(swiglu_bwd_kernel, dim3(grid_for(work)), dim3(256), 0, ft_stream(),
                       cptr<bf16_t>(da), cptr<bf16_t>(gu), mptr<bf16_t>(dgu), T, F);
  FT_LAUNCH_CHECK();
  return dgu;
}

TORCH_LIBRARY_FRAGMENT(ftamd, m) {
  m.def("swiglu_fwd(Tensor gu) -> Tensor", &swiglu_fwd);
  m.def("swiglu_bwd(Tensor da, Tensor gu) -> Tensor", &swiglu_bwd);
}
