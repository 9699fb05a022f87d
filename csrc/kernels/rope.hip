// Rotary position embedding, interleaved-pair convention, forward + backward.
//
// Parity: reference model.py:100-126 (`apply_rotary_emb`): adjacent pairs
// (x[2i], x[2i+1]) are treated as one complex number and multiplied by
// cis(pos * theta^(-2i/D)) in fp32, then cast back. The cos/sin tables are the
// reference's `precompute_freqs_cis` (model.py:51-71) split into real/imag
// planes (fp32 [S, D/2]); they are computed once on the host.
//
// Forward reads the fused QKV projection [T, (Hq+2Hkv)*D] and writes the rotated
// Q and K heads into a packed [T, (Hq+Hkv)*D] buffer that the flash-attention
// kernel reads directly (V is consumed from the QKV buffer in place, so the
// reference's repeat_kv copy (model.py:129-138) never exists). Backward rotates
// dQ/dK in place inside the fused dQKV gradient buffer. Each lane moves 8 elements
// (4 pairs): 16-B accesses for bf16 / fp16, 32 B for fp32 (--model-dtype).
#include "torch_utils.h"

namespace {

template <class E, bool BWD>
__global__ __launch_bounds__(256) void rope_kernel(const typename E::T* __restrict__ src, int src_stride,
                                                   typename E::T* __restrict__ dst, int dst_stride,
                                                   const float* __restrict__ cos_t,
                                                   const float* __restrict__ sin_t, int T, int S,
                                                   int width, int half_d) {
  // width = (Hq+Hkv)*D columns to rotate; each thread: 8 columns = 4 pairs
  const int vec_per_row = width >> 3;
  const long total = (long)T * vec_per_row;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total;
       i += (long)gridDim.x * blockDim.x) {
    const int row = (int)(i / vec_per_row);
    const int col = (int)(i - (long)row * vec_per_row) * 8;
    const int pos = row % S;
    const int fi = (col % (2 * half_d)) >> 1;  // pair index within the head
    const float4 c = *reinterpret_cast<const float4*>(cos_t + (long)pos * half_d + fi);
    const float4 s = *reinterpret_cast<const float4*>(sin_t + (long)pos * half_d + fi);
    float x[8], y[8];
    ld8<E>(src + (long)row * src_stride + col, x);
    const float cc[4] = {c.x, c.y, c.z, c.w};
    const float ss[4] = {BWD ? -s.x : s.x, BWD ? -s.y : s.y, BWD ? -s.z : s.z, BWD ? -s.w : s.w};
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const float a = x[2 * p], b = x[2 * p + 1];
      y[2 * p] = a * cc[p] - b * ss[p];
      y[2 * p + 1] = a * ss[p] + b * cc[p];
    }
    st8<E>(dst + (long)row * dst_stride + col, y);
  }
}

int grid_for(long work) {
  long g = (work + 255) / 256;
  return (int)std::max(1L, std::min(g, 256L * 16));
}

}  // namespace

// qkv: [T, (hq+2hkv)*d] -> qk: [T, (hq+hkv)*d] rotated
at::Tensor rope_fwd(const at::Tensor& qkv, const at::Tensor& cos_t, const at::Tensor& sin_t,
                    int64_t seq_len, int64_t hq, int64_t hkv, int64_t d) {
  FT_CHECK_CUDA(qkv);
  FT_CHECK_MODEL_DTYPE(qkv);
  FT_CHECK_CONTIG(qkv);
  FT_CHECK_F32(cos_t);
  FT_CHECK_F32(sin_t);
  TORCH_CHECK(d % 8 == 0, "rope: head_dim must be a multiple of 8");
  const int W = (hq + 2 * hkv) * d;
  TORCH_CHECK(qkv.size(-1) == W, "rope: qkv width mismatch");
  const int T = qkv.numel() / W;
  TORCH_CHECK(T % seq_len == 0, "rope: rows not a multiple of seq_len");
  TORCH_CHECK(cos_t.size(0) >= seq_len && cos_t.size(1) == d / 2, "rope: table shape");
  const at::DeviceGuard guard(qkv.device());
  const int width = (hq + hkv) * d;
  auto out = at::empty({T, width}, qkv.options());
  const long work = (long)T * (width / 8);
  if (work > 0)
    FT_DISPATCH_E(qkv.scalar_type(),
                  hipLaunchKernelGGL((rope_kernel<E, false>), dim3(grid_for(work)), dim3(256), 0, ft_stream(),
                                     cptr<typename E::T>(qkv), W, mptr<typename E::T>(out), width,
                                     cptr<float>(cos_t), cptr<float>(sin_t), T, (int)seq_len, width, (int)(d / 2)));
  FT_LAUNCH_CHECK();
  return out;
}

// In place on the first (hq+hkv)*d columns of dqkv [T, (hq+2hkv)*d].
void rope_bwd_(const at::Tensor& dqkv, const at::Tensor& cos_t, const at::Tensor& sin_t,
               int64_t seq_len, int64_t hq, int64_t hkv, int64_t d) {
  FT_CHECK_CUDA(dqkv);
  FT_CHECK_MODEL_DTYPE(dqkv);
  FT_CHECK_CONTIG(dqkv);
  const int W = (hq + 2 * hkv) * d;
  TORCH_CHECK(dqkv.size(-1) == W, "rope_bwd: width mismatch");
  const int T = dqkv.numel() / W;
  const int width = (hq + hkv) * d;
  const at::DeviceGuard guard(dqkv.device());
  const long work = (long)T * (width / 8);
  if (work > 0)
    FT_DISPATCH_E(dqkv.scalar_type(),
                  hipLaunchKernelGGL((rope_kernel<E, true>), dim3(grid_for(work)), dim3(256), 0, ft_stream(),
                                     cptr<typename E::T>(dqkv), W, mptr<typename E::T>(dqkv), W,
                                     cptr<float>(cos_t), cptr<float>(sin_t), T, (int)seq_len, width, (int)(d / 2)));
  FT_LAUNCH_CHECK();
}

TORCH_LIBRARY_FRAGMENT(ftamd, m) {
  m.def("rope_fwd(Tensor qkv, Tensor cos, Tensor sin, int seq_len, int hq, int hkv, int d) -> Tensor",
        &rope_fwd);
  m.def(
      "rope_bwd_(Tensor(a!) dqkv, Tensor cos, Tensor sin, int seq_len, int hq, int hkv, int d) -> ()",
      &rope_bwd_);
}
