// Token embedding gather (forward) and deterministic segment-sum backward.
//
// Parity: reference model.py:373 (`nn.Embedding` lookup). The backward replaces
// ATen's embedding_dense_backward: tokens are sorted once
// (stable, so each row's contributions are summed in a fixed order → bitwise
// reproducible, which the bit-exact resume test relies on), and one wave per
// distinct token sums its dy rows in fp32 and writes the bf16 gradient row
// straight into the flat gradient buffer. Rows never touched are zeroed by a
// memset of the embedding's gradient slice.
#include "torch_utils.h"

namespace {

__global__ __launch_bounds__(256) void emb_fwd_kernel(const int64_t* __restrict__ tok,
                                                      const bf16_t* __restrict__ w,
                                                      bf16_t* __restrict__ out, int T, int D) {
  const int row = blockIdx.x;
  const int64_t t = tok[row];
  const uint4* src = reinterpret_cast<const uint4*>(w + t * (long)D);
  uint4* dst = reinterpret_cast<uint4*>(out + (long)row * D);
  for (int c = threadIdx.x; c < D / 8; c += blockDim.x) dst[c] = src[c];
}

// sorted_tok[i], perm[i]: i-th smallest token and its original row.
__global__ __launch_bounds__(256) void emb_bwd_kernel(const int64_t* __restrict__ sorted_tok,
                                                      const int64_t* __restrict__ perm,
                                                      const bf16_t* __restrict__ dy,
                                                      bf16_t* __restrict__ dw, int T, int D,
                                                      bool accumulate) {
  const int wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (wave >= T) return;
  const int64_t t = sorted_tok[wave];
  if (wave > 0 && sorted_tok[wave - 1] == t) return;  // not the segment head
  int end = wave + 1;
  while (end < T && sorted_tok[end] == t) ++end;
  bf16_t* dst = dw + t * (long)D;
  for (int c = lane * 8; c < D; c += 64 * 8) {
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int k = wave; k < end; ++k) {
      float x[8];
      unpack8(*reinterpret_cast<const uint4*>(dy + perm[k] * (long)D + c), x);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += x[j];
    }
    if (accumulate) {
      float o[8];
      unpack8(*reinterpret_cast<const uint4*>(dst + c), o);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += o[j];
    }
    *reinterpret_cast<uint4*>(dst + c) = pack8(acc);
  }
}

}  // namespace

at::Tensor embedding_fwd(const at::Tensor& tokens, const at::Tensor& weight) {
  FT_CHECK_CUDA(weight);
  FT_CHECK_BF16(weight);
  FT_CHECK_CONTIG(weight);
  FT_CHECK_CONTIG(tokens);
  TORCH_CHECK(tokens.scalar_type() == at::kLong, "embedding: tokens must be int64");
  const int D = weight.size(1);
  TORCH_CHECK(D % 8 == 0, "embedding: dim must be a multiple of 8");
  const int T = tokens.numel();
  const at::DeviceGuard guard(weight.device());
  auto sizes = tokens.sizes().vec();
  sizes.push_back(D);
  auto out = at::empty(sizes, weight.options());
  if (T > 0)
    hipLaunchKernelGGL(emb_fwd_kernel, dim3(T), dim3(256), 0, ft_stream(), cptr<int64_t>(tokens),
                       cptr<bf16_t>(weight), mptr<bf16_t>(out), T, D);
  FT_LAUNCH_CHECK();
  return out;
}

// Writes (or accumulates) the dense gradient into dw [V, D].
void embedding_bwd_(const at::Tensor& dy, const at::Tensor& tokens, const at::Tensor& dw,
                    bool accumulate) {
  FT_CHECK_CUDA(dy);
  FT_CHECK_BF16(dy);
  FT_CHECK_CONTIG(dy);
  FT_CHECK_CONTIG(dw);
  const int D = dw.size(1);
  const int T = tokens.numel();
  TORCH_CHECK(dy.numel() == (long)T * D, "embedding_bwd: shape mismatch");
  const at::DeviceGuard guard(dw.device());
  auto flat = tokens.reshape({-1});
  auto sorted = at::sort(flat, /*stable=*/true, /*dim=*/0, /*descending=*/false);
  auto sorted_tok = std::get<0>(sorted).contiguous();
  auto perm = std::get<1>(sorted).contiguous();
  if (!accumulate) FT_HIP_CHECK(hipMemsetAsync(dw.data_ptr(), 0, dw.nbytes(), ft_stream()));
  if (T > 0) {
    const int blocks = (T * 64 + 255) / 256;
    hipLaunchKernelGGL(emb_bwd_kernel, dim3(blocks), dim3(256), 0, ft_stream(),
                       cptr<int64_t>(sorted_tok), cptr<int64_t>(perm), cptr<bf16_t>(dy),
                       mptr<bf16_t>(dw), T, D, accumulate);
  }
  FT_LAUNCH_CHECK();
}

TORCH_LIBRARY_FRAGMENT(ftamd, m) {
  m.def("embedding_fwd(Tensor tokens, Tensor weight) -> Tensor", &embedding_fwd);
  m.def("embedding_bwd_(Tensor dy, Tensor tokens, Tensor(a!) dw, bool accumulate) -> ()",
        &embedding_bwd_);
}
