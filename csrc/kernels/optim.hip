// Flat-buffer gradient L2 norm + clip + fused AdamW for gfx950.
//
// Parity:
//  * grad norm / clipping: reference utils.py:58-63 (`get_total_norm` with
//    error_if_nonfinite, then `clip_grads_with_norm_`). The reference's clip is a
//    silent no-op (generator consumed twice); here clipping is
//    real: coef = min(1, max_norm / (norm + 1e-6)) is computed on device and fed
//    to the optimizer without a host sync.
//  * AdamW: torch.optim.AdamW defaults used by the reference (train.py:68):
//    betas (0.9, 0.999), eps 1e-8, decoupled weight decay 0.01, bias correction.
//    Math in fp32, storage in the parameter/state dtype (bf16 by default like
//    the reference's all-bf16 states; fp16 / fp32 under --model-dtype, moments
//    optionally fp32). A non-finite norm skips the update for
//    every element (the host raises the reference's error path afterwards).
//
// The whole model's parameters, gradients and both moments each live in ONE
// flat buffer, so a step is two reduction launches + one streaming launch over
// ~8e9 elements instead of ~300-tensor foreach chains.
#include "torch_utils.h"

#include <vector>

#include <cstdlib>

namespace {

// 16-B vector access; NT = non-temporal (streaming) loads/stores: every byte of the
// optimizer pass is touched exactly once, so nothing is worth keeping in L2/MALL.
typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));

template <bool NT>
__device__ __forceinline__ uint4 ld16(const void* p) {
  if constexpr (NT) {
    const u32x4_t v = __builtin_nontemporal_load(reinterpret_cast<const u32x4_t*>(p));
    return make_uint4(v.x, v.y, v.z, v.w);
  } else {
    return *reinterpret_cast<const uint4*>(p);
  }
}

template <bool NT>
__device__ __forceinline__ void st16(void* p, uint4 v) {
  if constexpr (NT) {
    const u32x4_t w = {v.x, v.y, v.z, v.w};
    __builtin_nontemporal_store(w, reinterpret_cast<u32x4_t*>(p));
  } else {
    *reinterpret_cast<uint4*>(p) = v;
  }
}

// 8 elements of element type E (common.h) through 16-B (non-temporal) accesses.
template <class E, bool NT>
struct V8 {
  __device__ static void load(const typename E::T* p, float* f) {
    P8<E> r;
    r.v[0] = ld16<NT>(p);
    if constexpr (!E::is16) r.v[1] = ld16<NT>(p + 4);
    unp8<E>(r, f);
  }
  __device__ static void store(typename E::T* p, const float* f) {
    const P8<E> r = pk8<E>(f);
    st16<NT>(p, r.v[0]);
    if constexpr (!E::is16) st16<NT>(p + 4, r.v[1]);
  }
};

// Non-temporal loads/stores for the optimizer-pass kernels (plain ones measured slower:
// profiles/r1_stream_nt_ab.log).
bool stream_nt() { return true; }

constexpr int NORM_BLOCKS = 2048;

template <class G, bool NT>
__global__ __launch_bounds__(256) void sumsq_kernel(const typename G::T* __restrict__ g, long n8,
                                                    float* __restrict__ partial) {
  float s = 0.f;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n8; i += (long)gridDim.x * 256) {
    float x[8];
    V8<G, NT>::load(g + i * 8, x);
#pragma unroll
    for (int j = 0; j < 8; ++j) s += x[j] * x[j];
  }
  __shared__ float red[4];
  s = block_sum<256>(s, red);
  if (threadIdx.x == 0) partial[blockIdx.x] = s;
}

// stats[0] = ||g||, stats[1] = clip coefficient, stats[2] = 1 if non-finite.
// One 1024-thread block: the partial vector (tens of thousands of floats when the
// buckets' sums are taken during backward) is read with 16-B loads, so this
// serial step between backward and the optimizer stays a few microseconds.
__global__ __launch_bounds__(1024) void norm_finish_kernel(const float* __restrict__ partial,
                                                           int np, float extra_sumsq_scale,
                                                           float max_norm,
                                                           float* __restrict__ stats) {
  float s = 0.f;
  const int n4 = np >> 2;
  const float4* p4 = reinterpret_cast<const float4*>(partial);
  if ((reinterpret_cast<uintptr_t>(partial) & 15) == 0) {
    for (int i = threadIdx.x; i < n4; i += 1024) {
      const float4 v = p4[i];
      s += (v.x + v.y) + (v.z + v.w);
    }
    for (int i = 4 * n4 + threadIdx.x; i < np; i += 1024) s += partial[i];
  } else {
    for (int i = threadIdx.x; i < np; i += 1024) s += partial[i];
  }
  __shared__ float red[16];
  s = block_sum<1024>(s, red);
  if (threadIdx.x == 0) {
    const float norm = sqrtf(s * extra_sumsq_scale);
    stats[0] = norm;
    const bool bad = !isfinite(norm);
    stats[1] = (max_norm > 0.f && !bad) ? fminf(1.f, max_norm / (norm + 1e-6f)) : 1.f;
    // sticky: once a step's norm was non-finite every later update is skipped too, until
    // the host clears stats[2] (it only does so on an explicit reset). The trainer detects a
    // bad step two steps late without a host sync and rolls the counters back to it; the
    // parameters/moments are still exactly those before the bad step.
    stats[2] = (bad || stats[2] != 0.f) ? 1.f : 0.f;
  }
}

template <class P, class S, bool NT>
__global__ __launch_bounds__(256) void adamw_kernel(typename P::T* __restrict__ p,
                                                    const typename P::T* __restrict__ g,
                                                    typename S::T* __restrict__ m,
                                                    typename S::T* __restrict__ v,
                                                    long n8, float lr, float beta1, float beta2,
                                                    float eps, float wd, float inv_bc1,
                                                    float inv_sqrt_bc2,
                                                    const float* __restrict__ stats,
                                                    const float* __restrict__ hyper, int exact) {
  if (stats[2] != 0.f) return;  // non-finite gradient norm: skip the whole update
  if (hyper != nullptr) {
    // [lr, 1/bc1, 1/sqrt(bc2)] from device memory: a HIP-graph replay of the optimizer reads
    // this step's values (the host fills the buffer before the replay) instead of the
    // scalars baked in at capture
    lr = hyper[0];
    inv_bc1 = hyper[1];
    inv_sqrt_bc2 = hyper[2];
  }
  const float coef = stats[1];
  const float decay = 1.f - lr * wd;
  const float step = lr * inv_bc1;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n8; i += (long)gridDim.x * 256) {
    float pf[8], gf[8], mf[8], vf[8];
    V8<P, NT>::load(p + i * 8, pf);
    V8<P, NT>::load(g + i * 8, gf);
    V8<S, NT>::load(m + i * 8, mf);
    V8<S, NT>::load(v + i * 8, vf);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float gj = gf[j] * coef;
      pf[j] *= decay;
      mf[j] += (gj - mf[j]) * (1.f - beta1);
      vf[j] = vf[j] * beta2 + (1.f - beta2) * gj * gj;
      if (exact) {  // IEEE division / sqrt (FT_EXACT_MATH A/B)
        const float denom = sqrtf(vf[j]) * inv_sqrt_bc2 + eps;
        pf[j] -= step * mf[j] / denom;
      } else {
        const float denom = fast_sqrt(vf[j]) * inv_sqrt_bc2 + eps;
        pf[j] -= step * mf[j] * fast_rcp(denom);
      }
    }
    V8<P, NT>::store(p + i * 8, pf);
    V8<S, NT>::store(m + i * 8, mf);
    V8<S, NT>::store(v + i * 8, vf);
  }
}

// One 8-element vector per thread where possible: short-lived blocks keep more
// loads in flight than a capped grid-stride loop (5.9 vs 5.7 TB/s on MI355X,
// scripts/bw_bench.py); huge buffers still grid-stride.
int stream_grid(long n8) {
  long g = (n8 + 255) / 256;
  return (int)std::max(1L, std::min(g, 65535L));
}

void launch_sumsq(const at::Tensor& grad, long n8, int nb, float* partial) {
  const bool nt = stream_nt();
  FT_DISPATCH_E(grad.scalar_type(), {
    if (nt)
      hipLaunchKernelGGL((sumsq_kernel<E, true>), dim3(nb), dim3(256), 0, ft_stream(),
                         cptr<typename E::T>(grad), n8, partial);
    else
      hipLaunchKernelGGL((sumsq_kernel<E, false>), dim3(nb), dim3(256), 0, ft_stream(),
                         cptr<typename E::T>(grad), n8, partial);
  });
}

}  // namespace

// Writes [norm, coef, nonfinite] into stats (fp32[3], device).
void grad_norm_(const at::Tensor& grad, const at::Tensor& stats, double max_norm) {
  FT_CHECK_CUDA(grad);
  FT_CHECK_CONTIG(grad);
  FT_CHECK_F32(stats);
  TORCH_CHECK(grad.numel() % 8 == 0, "grad_norm: numel must be a multiple of 8");
  const at::DeviceGuard guard(grad.device());
  const long n8 = grad.numel() / 8;
  const int nb = std::max(1, std::min(NORM_BLOCKS, (int)((n8 + 255) / 256)));
  auto partial = at::empty({nb}, grad.options().dtype(at::kFloat));
  launch_sumsq(grad, n8, nb, mptr<float>(partial));
  FT_LAUNCH_CHECK();
  hipLaunchKernelGGL(norm_finish_kernel, dim3(1), dim3(1024), 0, ft_stream(), cptr<float>(partial), nb,
                     1.f, (float)max_norm, mptr<float>(stats));
  FT_LAUNCH_CHECK();
}

void adamw_(const at::Tensor& p, const at::Tensor& g, const at::Tensor& m, const at::Tensor& v,
            const at::Tensor& stats, double lr, double beta1, double beta2, double eps, double wd,
            int64_t step, int64_t max_blocks, const std::optional<at::Tensor>& hyper) {
  const float* hp = nullptr;
  if (hyper.has_value() && hyper->defined()) {
    FT_CHECK_F32((*hyper));
    TORCH_CHECK(hyper->is_cuda() && hyper->numel() >= 3, "adamw: hyper must be a device fp32[3]");
    hp = cptr<float>(*hyper);
  }
  FT_CHECK_CUDA(p);
  FT_CHECK_CONTIG(p);
  FT_CHECK_CONTIG(g);
  FT_CHECK_CONTIG(m);
  FT_CHECK_CONTIG(v);
  FT_CHECK_F32(stats);
  TORCH_CHECK(p.numel() == g.numel() && p.numel() == m.numel() && p.numel() == v.numel(),
              "adamw: size mismatch");
  TORCH_CHECK(p.numel() % 8 == 0, "adamw: numel must be a multiple of 8");
  TORCH_CHECK(p.scalar_type() == g.scalar_type() && m.scalar_type() == v.scalar_type(),
              "adamw: dtype mismatch");
  const at::DeviceGuard guard(p.device());
  const long n8 = p.numel() / 8;
  const float bc1 = 1.f - (float)std::pow(beta1, (double)step);
  const float bc2 = 1.f - (float)std::pow(beta2, (double)step);
  const float inv_bc1 = 1.f / bc1, inv_sqrt_bc2 = 1.f / std::sqrt(bc2);
  int nb = stream_grid(n8);
  // max_blocks > 0 overrides the default grid cap (both directions): small grids
  // leave CUs to a concurrent stream, large ones make every block short-lived so
  // the dispatcher can interleave a higher-priority stream's workgroups.
  if (max_blocks > 0) nb = (int)std::max(1L, std::min((n8 + 255) / 256, (long)max_blocks));
  const dim3 grid(nb), block(256);
  const bool nt = stream_nt();
  // parameter dtype P (= gradient dtype) in {bf16, fp16, fp32}; moments S either P or fp32
  TORCH_CHECK(m.scalar_type() == p.scalar_type() || m.scalar_type() == at::kFloat,
              "adamw: optimizer states must have the parameter dtype or fp32");
  // fp32 parameters (--model-dtype fp32) always take the IEEE division / square root: the
  // hardware v_rcp_f32 / v_sqrt_f32 (1 ulp) are below bf16/fp16 storage rounding but not below
  // fp32's, where torch AdamW's exact math is the parity target (docs/PARITY.md)
  const int exact = (int)ft_exact_math() || p.scalar_type() == at::kFloat;
  auto go = [&](auto ptag, auto stag) {
    using P = decltype(ptag);
    using S = decltype(stag);
    using PT = typename P::T;
    using ST = typename S::T;
    if (nt)
      hipLaunchKernelGGL((adamw_kernel<P, S, true>), grid, block, 0, ft_stream(), mptr<PT>(p),
                         cptr<PT>(g), mptr<ST>(m), mptr<ST>(v), n8, (float)lr, (float)beta1,
                         (float)beta2, (float)eps, (float)wd, inv_bc1, inv_sqrt_bc2,
                         cptr<float>(stats), hp, exact);
    else
      hipLaunchKernelGGL((adamw_kernel<P, S, false>), grid, block, 0, ft_stream(), mptr<PT>(p),
                         cptr<PT>(g), mptr<ST>(m), mptr<ST>(v), n8, (float)lr, (float)beta1,
                         (float)beta2, (float)eps, (float)wd, inv_bc1, inv_sqrt_bc2,
                         cptr<float>(stats), hp, exact);
  };
  FT_DISPATCH_E(p.scalar_type(), {
    if (m.scalar_type() == at::kFloat) go(E{}, EF32{});
    else go(E{}, E{});
  });
  FT_LAUNCH_CHECK();
}

// Per-bucket partial sums of squares, launched while backward is still running:
// block i of the launch writes partial[i] (grid = partial.numel()), so the total is
// a fixed-order sum independent of when each bucket finished (deterministic).
void sumsq_into_(const at::Tensor& grad, const at::Tensor& partial) {
  FT_CHECK_CUDA(grad);
  FT_CHECK_CONTIG(grad);
  FT_CHECK_F32(partial);
  FT_CHECK_CONTIG(partial);
  TORCH_CHECK(grad.numel() % 8 == 0, "sumsq_into: numel must be a multiple of 8");
  TORCH_CHECK(partial.numel() >= 1 && partial.numel() <= 65535, "sumsq_into: bad partial size");
  const at::DeviceGuard guard(grad.device());
  const long n8 = grad.numel() / 8;
  const int nb = (int)partial.numel();
  launch_sumsq(grad, n8, nb, mptr<float>(partial));
  FT_LAUNCH_CHECK();
}

// stats = [norm, clip coef, nonfinite] from a vector of partial sums of squares.
void norm_finish_(const at::Tensor& partial, const at::Tensor& stats, double max_norm) {
  FT_CHECK_CUDA(partial);
  FT_CHECK_F32(partial);
  FT_CHECK_F32(stats);
  const at::DeviceGuard guard(partial.device());
  hipLaunchKernelGGL(norm_finish_kernel, dim3(1), dim3(1024), 0, ft_stream(), cptr<float>(partial),
                     (int)partial.numel(), 1.f, (float)max_norm, mptr<float>(stats));
  FT_LAUNCH_CHECK();
}

// A stream whose kernels dispatch only to every `stride`-th CU (hipExtStreamCreateWithCUMask), for
// confining the optimizer's memory-bound AdamW launches to a slice of the chip while the next
// forward's GEMMs keep the rest (scripts/ab_step.py knob cumask). Returns the hipStream_t as an
// integer for torch.cuda.ExternalStream; the stream lives for the process.
int64_t cu_masked_stream(int64_t stride, int64_t phase) {
  TORCH_CHECK(stride >= 1 && phase >= 0 && phase < stride, "cu_masked_stream: 0 <= phase < stride");
  int dev = 0, ncu = 0;
  FT_HIP_CHECK(hipGetDevice(&dev));
  FT_HIP_CHECK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
  std::vector<uint32_t> mask((ncu + 31) / 32, 0u);
  for (int c = (int)phase; c < ncu; c += (int)stride) mask[c / 32] |= 1u << (c % 32);
  hipStream_t st = nullptr;
  FT_HIP_CHECK(hipExtStreamCreateWithCUMask(&st, (uint32_t)mask.size(), mask.data()));
  return reinterpret_cast<int64_t>(st);
}

TORCH_LIBRARY_FRAGMENT(ftamd, m) {
  m.def("cu_masked_stream(int stride, int phase=0) -> int", &cu_masked_stream);
  m.def("sumsq_into_(Tensor grad, Tensor(a!) partial) -> ()", &sumsq_into_);
  m.def("norm_finish_(Tensor partial, Tensor(a!) stats, float max_norm) -> ()", &norm_finish_);
  m.def("grad_norm_(Tensor grad, Tensor(a!) stats, float max_norm) -> ()", &grad_norm_);
  m.def(
      "adamw_(Tensor(a!) p, Tensor g, Tensor(b!) m, Tensor(c!) v, Tensor stats, float lr, float "
      "beta1, float beta2, float eps, float wd, int step, int max_blocks=0, Tensor? hyper=None) -> ()",
      &adamw_);
}
