// Bandwidth-bound bf16 2-D transpose for gfx950: out[C, R] = x[R, C]^T.
//
// Why: the weight-gradient GEMM dW[N, K] = dY^T X reduces over tokens, and with
// row-major activations both operands are token-major ("NT"); hipBLASLt runs that
// layout at ~0.9-1.1 PF on MI355X but the K-contiguous "TN" layout of the same
// product at ~1.15-1.45 PF (scripts/gemm_layout_bench.py, profiles/). Transposing
// the two operands costs one read + one write each, far less than the GEMM time
// it saves for the big projections (w13, w2, LM head).
//
// Tile 64 x 64 per 256-thread block: each lane loads two 16-B row segments
// (8 bf16), stages them in LDS with a 2-element row pad (bank-conflict-light
// column reads), and writes two 16-B segments of the transposed rows. Both the
// global loads and the stores are full 128-B lines per 8 lanes.
#include "torch_utils.h"

namespace {

constexpr int TT = 64;
constexpr int PAD = 2;

__global__ __launch_bounds__(256) void transpose_kernel(const bf16_t* __restrict__ x,
                                                        bf16_t* __restrict__ out, int R, int C) {
  __shared__ bf16_t tile[TT][TT + PAD];
  const int tilesC = C / TT;
  const int tr = blockIdx.x / tilesC, tc = blockIdx.x % tilesC;
  const int r0 = tr * TT, c0 = tc * TT;
  const int t = threadIdx.x;
  // load: 64 rows x 8 segments of 8 bf16
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int id = t + k * 256;
    const int row = id >> 3, seg = id & 7;
    const uint4 v = *reinterpret_cast<const uint4*>(x + (size_t)(r0 + row) * C + c0 + seg * 8);
    const bf16_t* e = reinterpret_cast<const bf16_t*>(&v);
#pragma unroll
    for (int j = 0; j < 8; ++j) tile[row][seg * 8 + j] = e[j];
  }
  __syncthreads();
  // store: output row = input column c (64 of them), 8 segments of 8 input rows
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int id = t + k * 256;
    const int c = id >> 3, seg = id & 7;
    uint4 v;
    bf16_t* e = reinterpret_cast<bf16_t*>(&v);
#pragma unroll
    for (int j = 0; j < 8; ++j) e[j] = tile[seg * 8 + j][c];
    *reinterpret_cast<uint4*>(out + (size_t)(c0 + c) * R + r0 + seg * 8) = v;
  }
}

}  // namespace

// out (optional, [C, R]) = x^T for a contiguous 2-D bf16 x with R, C multiples of 64.
at::Tensor transpose2d(const at::Tensor& x, const std::optional<at::Tensor>& out_opt) {
  FT_CHECK_CUDA(x);
  FT_CHECK_BF16(x);
  FT_CHECK_CONTIG(x);
  TORCH_CHECK(x.dim() == 2, "transpose2d: 2-D input expected");
  const int R = x.size(0), C = x.size(1);
  TORCH_CHECK(R % TT == 0 && C % TT == 0, "transpose2d: dims must be multiples of 64");
  at::Tensor out = out_opt.has_value() && out_opt->defined() ? *out_opt : at::empty({C, R}, x.options());
  FT_CHECK_CONTIG(out);
  TORCH_CHECK(out.numel() == x.numel(), "transpose2d: out size");
  const at::DeviceGuard guard(x.device());
  const long blocks = (long)(R / TT) * (C / TT);
  if (blocks > 0) {
    hipLaunchKernelGGL(transpose_kernel, dim3((unsigned)blocks), dim3(256), 0, ft_stream(),
                       cptr<bf16_t>(x), mptr<bf16_t>(out), R, C);
    FT_LAUNCH_CHECK();
  }
  return out;
}

TORCH_LIBRARY_FRAGMENT(ftamd, m) {
  m.def("transpose2d(Tensor x, Tensor? out=None) -> Tensor", &transpose2d);
}
