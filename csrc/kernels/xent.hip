// Fused vocabulary cross-entropy, forward + backward, on bf16 (fp16 / fp32) logits.
//
// Parity: reference train.py:101-102
//   loss = cross_entropy(logits.flatten(0,1).float(), labels, reduction="sum") / num_items
// with ignore_index = -100 (labels masked by the collator, dataset.py:50).
// The reference materialises an fp32 copy of the [T, V] logits (1 GiB at
// T=2048, V=131072) plus its gradient; here the bf16 logits are read once in
// forward (online max/log-sum-exp per row, fp32 accumulation) and once in
// backward, which overwrites them in place with dlogits = (softmax - onehot) *
// grad * inv_count in bf16. One 256-thread block per row, 16-B loads.
#include "torch_utils.h"

namespace {

constexpr float LOG2E = 1.4426950408889634f;

template <class E>
__global__ __launch_bounds__(256) void xent_fwd_kernel(const typename E::T* __restrict__ logits,
                                                       const int64_t* __restrict__ labels,
                                                       float* __restrict__ loss,
                                                       float* __restrict__ lse, int V,
                                                       int ignore_index) {
  const int row = blockIdx.x;
  const typename E::T* lr = logits + (long)row * V;
  float m = -INFINITY, s = 0.f;
  for (int c = threadIdx.x * 8; c < V; c += 256 * 8) {
    float x[8];
    ld8<E>(lr + c, x);
    float lm = x[0];
#pragma unroll
    for (int j = 1; j < 8; ++j) lm = fmaxf(lm, x[j]);
    const float nm = fmaxf(m, lm);
    float acc = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) acc += exp2f((x[j] - nm) * LOG2E);
    s = s * exp2f((m - nm) * LOG2E) + acc;
    m = nm;
  }
  // wave-level merge of (m, s)
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float om = __shfl_xor(m, o, 64), os = __shfl_xor(s, o, 64);
    const float nm = fmaxf(m, om);
    s = (m == -INFINITY ? 0.f : s * exp2f((m - nm) * LOG2E)) +
        (om == -INFINITY ? 0.f : os * exp2f((om - nm) * LOG2E));
    m = nm;
  }
  __shared__ float sm[4], ssum[4];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) {
    sm[wid] = m;
    ssum[wid] = s;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float M = sm[0];
    for (int i = 1; i < 4; ++i) M = fmaxf(M, sm[i]);
    float S = 0.f;
    for (int i = 0; i < 4; ++i) S += ssum[i] * exp2f((sm[i] - M) * LOG2E);
    const float l = M + logf(S);
    lse[row] = l;
    const int64_t y = labels[row];
    loss[row] = (y == ignore_index) ? 0.f : (l - ld1<E>(lr + y));
  }
}

// dlogits in place: (exp(x - lse) - [j == y]) * scale, scale = grad * inv_count.
template <class E>
__global__ __launch_bounds__(256) void xent_bwd_kernel(typename E::T* __restrict__ logits,
                                                       const int64_t* __restrict__ labels,
                                                       const float* __restrict__ lse,
                                                       const float* __restrict__ grad,
                                                       const float* __restrict__ inv_count, int V,
                                                       int T, int ignore_index) {
  // rows grid-strided over y (gridDim.y is capped below 65536; long-context T exceeds it)
  for (int row = blockIdx.y; row < T; row += gridDim.y) {
    const int64_t y = labels[row];
    typename E::T* lr = logits + (long)row * V;
    const float scale = (y == ignore_index) ? 0.f : grad[0] * inv_count[0];
    const float l = lse[row];
    for (int c = (blockIdx.x * 256 + threadIdx.x) * 8; c < V; c += gridDim.x * 256 * 8) {
      float x[8];
      ld8<E>(lr + c, x);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float p = exp2f((x[j] - l) * LOG2E);
        if (c + j == y) p -= 1.f;
        x[j] = p * scale;
      }
      st8<E>(lr + c, x);
    }
  }
}

// x *= g[0] unless g[0] == 1 (then every block exits at once): the upstream gradient of a
// loss whose input gradients were already formed in the forward pass (fused LM head).
template <class E>
__global__ __launch_bounds__(256) void scale_by_kernel(typename E::T* __restrict__ x, long n8,
                                                       const float* __restrict__ g) {
  const float s = g[0];
  if (s == 1.f) return;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n8; i += (long)gridDim.x * 256) {
    float v[8];
    ld8<E>(x + i * 8, v);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] *= s;
    st8<E>(x + i * 8, v);
  }
}

}  // namespace

void scale_by_(const at::Tensor& x, const at::Tensor& g) {
  FT_CHECK_CUDA(x);
  FT_CHECK_MODEL_DTYPE(x);
  FT_CHECK_CONTIG(x);
  FT_CHECK_F32(g);
  TORCH_CHECK(x.numel() % 8 == 0, "scale_by_: numel must be a multiple of 8");
  const at::DeviceGuard guard(x.device());
  const long n8 = x.numel() / 8;
  if (n8 > 0)
    FT_DISPATCH_E(x.scalar_type(),
                  hipLaunchKernelGGL(scale_by_kernel<E>, dim3((unsigned)std::min<long>((n8 + 255) / 256, 2048)),
                                     dim3(256), 0, ft_stream(), mptr<typename E::T>(x), n8, cptr<float>(g)));
  FT_LAUNCH_CHECK();
}

// Returns (per-row loss [T] fp32, lse [T] fp32).
std::tuple<at::Tensor, at::Tensor> xent_fwd(const at::Tensor& logits, const at::Tensor& labels,
                                            int64_t ignore_index) {
  FT_CHECK_CUDA(logits);
  FT_CHECK_MODEL_DTYPE(logits);
  FT_CHECK_CONTIG(logits);
  FT_CHECK_CONTIG(labels);
  TORCH_CHECK(labels.scalar_type() == at::kLong, "xent: labels must be int64");
  const int V = logits.size(-1);
  TORCH_CHECK(V % 8 == 0, "xent: vocab must be a multiple of 8");
  const int T = logits.numel() / V;
  TORCH_CHECK(labels.numel() == T, "xent: labels shape mismatch");
  const at::DeviceGuard guard(logits.device());
  auto loss = at::empty({T}, logits.options().dtype(at::kFloat));
  auto lse = at::empty({T}, logits.options().dtype(at::kFloat));
  if (T > 0)
    FT_DISPATCH_E(logits.scalar_type(),
                  hipLaunchKernelGGL(xent_fwd_kernel<E>, dim3(T), dim3(256), 0, ft_stream(),
                                     cptr<typename E::T>(logits), cptr<int64_t>(labels), mptr<float>(loss),
                                     mptr<float>(lse), V, (int)ignore_index));
  FT_LAUNCH_CHECK();
  return {loss, lse};
}

// Overwrites `logits` with dlogits. grad and inv_count are 1-element fp32 device tensors.
void xent_bwd_(const at::Tensor& logits, const at::Tensor& labels, const at::Tensor& lse,
               const at::Tensor& grad, const at::Tensor& inv_count, int64_t ignore_index) {
  FT_CHECK_CUDA(logits);
  FT_CHECK_MODEL_DTYPE(logits);
  FT_CHECK_CONTIG(logits);
  FT_CHECK_F32(grad);
  FT_CHECK_F32(inv_count);
  const int V = logits.size(-1);
  const int T = logits.numel() / V;
  const at::DeviceGuard guard(logits.device());
  const int bx = std::max(1, std::min((V / 8 + 255) / 256, 8));
  if (T > 0)
    FT_DISPATCH_E(logits.scalar_type(),
                  hipLaunchKernelGGL(xent_bwd_kernel<E>, dim3(bx, std::min(T, 32768)), dim3(256), 0, ft_stream(),
                                     mptr<typename E::T>(logits), cptr<int64_t>(labels), cptr<float>(lse),
                                     cptr<float>(grad), cptr<float>(inv_count), V, T, (int)ignore_index));
  FT_LAUNCH_CHECK();
}

TORCH_LIBRARY_FRAGMENT(ftamd, m) {
  m.def("scale_by_(Tensor(a!) x, Tensor g) -> ()", &scale_by_);
  m.def("xent_fwd(Tensor logits, Tensor labels, int ignore_index) -> (Tensor, Tensor)", &xent_fwd);
  m.def(
      "xent_bwd_(Tensor(a!) logits, Tensor labels, Tensor lse, Tensor grad, Tensor inv_count, int "
      "ignore_index) -> ()",
      &xent_bwd_);
}
