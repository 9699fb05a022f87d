// SwiGLU activation on the fused up/gate projection, forward + backward.
//
// Parity: reference model.py:253-254 `w2(silu(w1 x) * w3 x)`. The two input
// projections run as ONE GEMM against the concatenated [w1; w3] weight (they
// are adjacent in the flat parameter buffer), so this kernel reads gu =
// [T, 2F] (gate in columns [0,F), up in [F,2F)) and writes a = silu(g) * u.
// fp32 math, one rounding per output (the reference rounds twice). bf16 / fp16 / fp32
// (--model-dtype); 16-B (32-B for fp32) vector accesses, grid-stride. The tiled variants
// that also write the transposed outputs are bf16 (the default model dtype's dW layout).
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

// Tiled variants that also write the transposed output, which the weight-gradient
// GEMMs consume in their fast K-contiguous ("TN") layout: one 64 x 64 tile per block,
// the transpose goes through LDS, both stores are 16-B vectors. Saves the separate
// transpose kernel's full read of the activation (ops/functional.py: weight_grad).
constexpr int TT = 64;

__global__ __launch_bounds__(256) void swiglu_fwd_t_kernel(const bf16_t* __restrict__ gu,
                                                           bf16_t* __restrict__ a,
                                                           bf16_t* __restrict__ aT, int T, int F, int exact) {
  __shared__ bf16_t tile[TT][TT + 2];
  const int tilesF = F / TT;
  const int r0 = (blockIdx.x / tilesF) * TT, c0 = (blockIdx.x % tilesF) * TT;
  const int t = threadIdx.x;
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int id = t + k * 256, row = id >> 3, seg = id & 7;
    const long base = (long)(r0 + row) * 2 * F + c0 + seg * 8;
    float g[8], u[8], o[8];
    unpack8(*reinterpret_cast<const uint4*>(gu + base), g);
    unpack8(*reinterpret_cast<const uint4*>(gu + base + F), u);
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = g[j] * sigmoid_f(g[j], exact) * u[j];
    const uint4 v = pack8(o);
    if (a != nullptr) *reinterpret_cast<uint4*>(a + (long)(r0 + row) * F + c0 + seg * 8) = v;
    const bf16_t* e = reinterpret_cast<const bf16_t*>(&v);
#pragma unroll
    for (int j = 0; j < 8; ++j) tile[row][seg * 8 + j] = e[j];
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int id = t + k * 256, c = id >> 3, seg = id & 7;
    uint4 v;
    bf16_t* e = reinterpret_cast<bf16_t*>(&v);
#pragma unroll
    for (int j = 0; j < 8; ++j) e[j] = tile[seg * 8 + j][c];
    *reinterpret_cast<uint4*>(aT + (long)(c0 + c) * T + r0 + seg * 8) = v;
  }
}

// Backward with the transposed output: a wave owns a 64-token x 64-feature tile; lane (tg = lane & 7, fc = lane >> 3)
// owns tokens 8 tg .. 8 tg + 7 x features 8 fc .. 8 fc + 7 and transposes that 8 x 8 block in
// registers. Every access is a 16-B vector and the 8 lanes of one tg (loads, row-major stores)
// or of one fc (transposed stores) cover 128 contiguous bytes: no LDS, no 2-byte LDS traffic
// (92.3 vs 96.5 us for the LDS-tiled form at 2048 x 14336; profiles/r2_kernel_bandwidth.md).
__global__ __launch_bounds__(256) void swiglu_bwd_rt_kernel(const bf16_t* __restrict__ da,
                                                            const bf16_t* __restrict__ gu,
                                                            bf16_t* __restrict__ dgu,
                                                            bf16_t* __restrict__ dguT, int T, int F, int exact) {
  const int lane = threadIdx.x & 63;
  const int tilesF = F / TT;
  const int tile = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (tile >= (T / TT) * tilesF) return;  // wave-uniform
  const int tok0 = (tile / tilesF) * TT + (lane & 7) * 8;
  const int f0 = (tile % tilesF) * TT + (lane >> 3) * 8;
  uint4 G[8], U[8], D[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const long rb = (long)(tok0 + i) * 2 * F + f0;
    G[i] = *reinterpret_cast<const uint4*>(gu + rb);
    U[i] = *reinterpret_cast<const uint4*>(gu + rb + F);
    D[i] = *reinterpret_cast<const uint4*>(da + (long)(tok0 + i) * F + f0);
  }
  bf16_t og[8][8], ou[8][8];  // [token][feature]
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    float g[8], u[8], d[8], dg[8], du[8];
    unpack8(G[i], g);
    unpack8(U[i], u);
    unpack8(D[i], d);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      swiglu_grad(g[j], u[j], d[j], exact, dg[j], du[j]);
      og[i][j] = f2bf(dg[j]);
      ou[i][j] = f2bf(du[j]);
    }
    if (dgu != nullptr) {
      const long rb = (long)(tok0 + i) * 2 * F + f0;
      *reinterpret_cast<uint4*>(dgu + rb) = pack8(dg);
      *reinterpret_cast<uint4*>(dgu + rb + F) = pack8(du);
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    uint4 vg, vu;
    vg.x = og[0][j] | ((uint32_t)og[1][j] << 16);
    vg.y = og[2][j] | ((uint32_t)og[3][j] << 16);
    vg.z = og[4][j] | ((uint32_t)og[5][j] << 16);
    vg.w = og[6][j] | ((uint32_t)og[7][j] << 16);
    vu.x = ou[0][j] | ((uint32_t)ou[1][j] << 16);
    vu.y = ou[2][j] | ((uint32_t)ou[3][j] << 16);
    vu.z = ou[4][j] | ((uint32_t)ou[5][j] << 16);
    vu.w = ou[6][j] | ((uint32_t)ou[7][j] << 16);
    *reinterpret_cast<uint4*>(dguT + (long)(f0 + j) * T + tok0) = vg;
    *reinterpret_cast<uint4*>(dguT + (long)(F + f0 + j) * T + tok0) = vu;
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

// (a [T, F], a^T [F, T]); T and F multiples of 64. plain=false: only a^T is written
// (a is returned empty) for consumers that read the activation transposed.
std::tuple<at::Tensor, at::Tensor> swiglu_fwd_t(const at::Tensor& gu, bool plain) {
  FT_CHECK_CUDA(gu);
  FT_CHECK_BF16(gu);
  FT_CHECK_CONTIG(gu);
  const int F = gu.size(-1) / 2;
  const int T = gu.numel() / (2 * F);
  TORCH_CHECK(F % TT == 0 && T % TT == 0, "swiglu_fwd_t: T and F must be multiples of 64");
  const at::DeviceGuard guard(gu.device());
  auto a = plain ? at::empty({T, F}, gu.options()) : at::empty({0}, gu.options());
  auto aT = at::empty({F, T}, gu.options());
  if (T > 0)
    hipLaunchKernelGGL(swiglu_fwd_t_kernel, dim3((T / TT) * (F / TT)), dim3(256), 0, ft_stream(),
                       cptr<bf16_t>(gu), plain ? mptr<bf16_t>(a) : nullptr, mptr<bf16_t>(aT), T, F,
                       (int)ft_exact_math());
  FT_LAUNCH_CHECK();
  return {a, aT};
}

// (dgu [T, 2F], dgu^T [2F, T]); T and F multiples of 64. plain=false: only dgu^T.
std::tuple<at::Tensor, at::Tensor> swiglu_bwd_t(const at::Tensor& da, const at::Tensor& gu, bool plain) {
  FT_CHECK_CUDA(gu);
  FT_CHECK_BF16(gu);
  FT_CHECK_CONTIG(gu);
  FT_CHECK_CONTIG(da);
  const int F = gu.size(-1) / 2;
  const int T = gu.numel() / (2 * F);
  TORCH_CHECK(da.numel() == (long)T * F, "swiglu_bwd_t: shape mismatch");
  TORCH_CHECK(F % TT == 0 && T % TT == 0, "swiglu_bwd_t: T and F must be multiples of 64");
  const at::DeviceGuard guard(gu.device());
  auto dgu = plain ? at::empty({T, 2 * F}, gu.options()) : at::empty({0}, gu.options());
  auto dguT = at::empty({2 * F, T}, gu.options());
  const int tiles = (T / TT) * (F / TT);
  if (T > 0)
    hipLaunchKernelGGL(swiglu_bwd_rt_kernel, dim3((tiles + 3) / 4), dim3(256), 0, ft_stream(),
                       cptr<bf16_t>(da), cptr<bf16_t>(gu), plain ? mptr<bf16_t>(dgu) : nullptr,
                       mptr<bf16_t>(dguT), T, F, (int)ft_exact_math());
  FT_LAUNCH_CHECK();
  return {dgu, dguT};
}

// Same-process A/B of the IEEE-exact vs hardware reciprocal / sqrt (see ft_exact_math).
void set_exact_math(bool on) { ft_exact_math() = on; }

TORCH_LIBRARY_FRAGMENT(ftamd, m) {
  m.def("set_exact_math(bool on) -> ()", &set_exact_math);
  m.def("swiglu_fwd_t(Tensor gu, bool plain=True) -> (Tensor, Tensor)", &swiglu_fwd_t);
  m.def("swiglu_bwd_t(Tensor da, Tensor gu, bool plain=True) -> (Tensor, Tensor)", &swiglu_bwd_t);
  m.def("swiglu_fwd(Tensor gu) -> Tensor", &swiglu_fwd);
  m.def("swiglu_bwd(Tensor da, Tensor gu) -> Tensor", &swiglu_bwd);
}
