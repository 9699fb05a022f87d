// Token embedding gather (forward) and deterministic segment-sum backward.
//
// Parity: reference model.py:373 (`nn.Embedding` lookup). The backward replaces
// ATen's embedding_dense_backward: tokens are sorted once
// (stable, so each row's contributions are summed in a fixed order → bitwise
// reproducible, which the bit-exact resume test relies on), and one wave per
// distinct token sums its dy rows in fp32 and writes the bf16 gradient row
// straight into the flat gradient buffer. Rows never touched are zeroed by a
// memset of the embedding's gradient slice.
//
// The sort is in-tree (no ATen/rocPRIM kernel on the path): one 1024-thread workgroup
// runs a stable LSD radix sort with 6-bit digits (3 passes for a 131072-token vocabulary)
// over the B*S token ids (2048 per GPU; 16384 after the DP sparse exchange gathers 8
// ranks). Per pass: a digit histogram (LDS atomics: counts are order-independent),
// then rounds of 1024 keys in index order; inside a wave, lanes with the same digit find
// each other with six ballots and rank themselves by lane (popcount of the lower lanes'
// match mask), wave counts are prefix-summed across the 16 waves per digit, and every key
// goes to bin start + earlier rounds + earlier waves + its rank — i.e. stably.
#include "torch_utils.h"

#include <algorithm>

namespace {

// row copy in 16-B vectors (any element size; rows are whole vectors)
__global__ __launch_bounds__(256) void emb_fwd_kernel(const int64_t* __restrict__ tok,
                                                      const char* __restrict__ w,
                                                      char* __restrict__ out, int T, int row_bytes) {
  const int row = blockIdx.x;
  const int64_t t = tok[row];
  const uint4* src = reinterpret_cast<const uint4*>(w + t * (long)row_bytes);
  uint4* dst = reinterpret_cast<uint4*>(out + (long)row * row_bytes);
  for (int c = threadIdx.x; c < row_bytes / 16; c += blockDim.x) dst[c] = src[c];
}

constexpr int SORT_NT = 1024, SORT_W = SORT_NT / 64, SORT_BITS = 6, SORT_BINS = 1 << SORT_BITS;

// Stable LSD radix sort of tok[0..T) (values < 2^(6*passes)) with the row index as payload.
// Pass p reads (p == 0 ? tok, iota : buffer (p-1)&1) and writes buffer p&1 (k[2][T], v[2][T]).
__global__ __launch_bounds__(SORT_NT) void tok_sort_kernel(const int64_t* __restrict__ tok, int T, int passes,
                                                           int* __restrict__ keys, int* __restrict__ vals) {
  __shared__ int hist[SORT_BINS];
  __shared__ int start[SORT_BINS];
  __shared__ int rbase[SORT_BINS];
  __shared__ int wcnt[SORT_W][SORT_BINS];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const unsigned long long lower = (1ull << lane) - 1ull;
  for (int pass = 0; pass < passes; ++pass) {
    const int shift = pass * SORT_BITS;
    const int* sk = pass == 0 ? nullptr : keys + ((pass - 1) & 1) * (long)T;
    const int* sv = pass == 0 ? nullptr : vals + ((pass - 1) & 1) * (long)T;
    int* dk = keys + (pass & 1) * (long)T;
    int* dv = vals + (pass & 1) * (long)T;
    if (tid < SORT_BINS) hist[tid] = 0;
    __syncthreads();
    for (int i = tid; i < T; i += SORT_NT) {
      const int k = sk ? sk[i] : (int)tok[i];
      atomicAdd(&hist[(k >> shift) & (SORT_BINS - 1)], 1);
    }
    __syncthreads();
    if (tid == 0) {
      int s = 0;
      for (int b = 0; b < SORT_BINS; ++b) {
        start[b] = s;
        s += hist[b];
      }
    }
    for (int base = 0; base < T; base += SORT_NT) {
      const int i = base + tid;
      const bool valid = i < T;
      const int k = valid ? (sk ? sk[i] : (int)tok[i]) : 0;
      const int v = valid ? (sk ? sv[i] : i) : 0;
      const int d = (k >> shift) & (SORT_BINS - 1);
      unsigned long long m = __ballot(valid);
#pragma unroll
      for (int b = 0; b < SORT_BITS; ++b) {
        const unsigned long long bb = __ballot(valid && ((d >> b) & 1));
        m &= ((d >> b) & 1) ? bb : ~bb;
      }
      const int rank = __popcll(m & lower);
      wcnt[wid][lane] = 0;
      __syncthreads();
      if (valid && rank == 0) wcnt[wid][d] = __popcll(m);
      __syncthreads();
      if (tid < SORT_BINS) {  // exclusive prefix over the waves, per digit
        int s = 0;
        for (int w = 0; w < SORT_W; ++w) {
          const int c = wcnt[w][tid];
          wcnt[w][tid] = s;
          s += c;
        }
        rbase[tid] = start[tid];
        start[tid] += s;
      }
      __syncthreads();
      if (valid) {
        const int pos = rbase[d] + wcnt[wid][d] + rank;
        dk[pos] = k;
        dv[pos] = v;
      }
      __syncthreads();  // (also orders this pass's global writes before the next pass's reads)
    }
  }
}

// sorted_tok[i], perm[i]: i-th smallest token and its original row.
template <class E>
__global__ __launch_bounds__(256) void emb_bwd_kernel(const int* __restrict__ sorted_tok,
                                                      const int* __restrict__ perm,
                                                      const typename E::T* __restrict__ dy,
                                                      typename E::T* __restrict__ dw, int T, int D,
                                                      bool accumulate) {
  const int wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (wave >= T) return;
  const int t = sorted_tok[wave];
  if (wave > 0 && sorted_tok[wave - 1] == t) return;  // not the segment head
  int end = wave + 1;
  while (end < T && sorted_tok[end] == t) ++end;
  typename E::T* dst = dw + t * (long)D;
  for (int c = lane * 8; c < D; c += 64 * 8) {
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int k = wave; k < end; ++k) {
      float x[8];
      ld8<E>(dy + perm[k] * (long)D + c, x);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += x[j];
    }
    if (accumulate) {
      float o[8];
      ld8<E>(dst + c, o);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += o[j];
    }
    st8<E>(dst + c, acc);
  }
}

// emb_bwd_kernel for a fresh (zeroed) gradient, plus the gradient-norm partials of what it stores:
// every row it does not write is zero, so the sum of squares of the whole [V, D] gradient is the
// sum over the written rows — no pass over the 1 GB buffer (the 8B vocabulary). Block b takes
// segment waves b*4 .. in a grid-stride loop, each lane its columns in a fixed order, and writes
// part[b]; the remaining partial slots are zeroed. Fixed order throughout: deterministic.
template <class E>
__global__ __launch_bounds__(256) void emb_bwd_sq_kernel(const int* __restrict__ sorted_tok,
                                                         const int* __restrict__ perm,
                                                         const typename E::T* __restrict__ dy,
                                                         typename E::T* __restrict__ dw, int T, int D,
                                                         float* __restrict__ part, int nparts) {
  __shared__ float red[4];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  float sq = 0.f;
  for (int wave = blockIdx.x * 4 + wid; wave < T; wave += gridDim.x * 4) {
    const int t = sorted_tok[wave];
    if (wave > 0 && sorted_tok[wave - 1] == t) continue;  // not the segment head
    int end = wave + 1;
    while (end < T && sorted_tok[end] == t) ++end;
    typename E::T* dst = dw + t * (long)D;
    for (int c = lane * 8; c < D; c += 64 * 8) {
      float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
      for (int k = wave; k < end; ++k) {
        float x[8];
        ld8<E>(dy + perm[k] * (long)D + c, x);
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] += x[j];
      }
      const P8<E> r = pk8<E>(acc);
      *reinterpret_cast<uint4*>(dst + c) = r.v[0];
      if constexpr (!E::is16) *reinterpret_cast<uint4*>(dst + c + 4) = r.v[1];
      float st[8];
      unp8<E>(r, st);  // the stored (rounded) values
#pragma unroll
      for (int j = 0; j < 8; ++j) sq = fmaf(st[j], st[j], sq);
    }
  }
  const float tot = block_sum<256>(sq, red);
  if (threadIdx.x == 0) part[blockIdx.x] = tot;
  for (long i = blockIdx.x + (long)gridDim.x * (1 + threadIdx.x); i < nparts; i += (long)gridDim.x * 256)
    part[i] = 0.f;
}

}  // namespace

at::Tensor embedding_fwd(const at::Tensor& tokens, const at::Tensor& weight) {
  FT_CHECK_CUDA(weight);
  FT_CHECK_MODEL_DTYPE(weight);
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
                       cptr<char>(weight), mptr<char>(out), T, (int)(D * weight.element_size()));
  FT_LAUNCH_CHECK();
  return out;
}

// Writes (or accumulates) the dense gradient into dw [V, D]. part (fp32, not accumulating): also
// the gradient-norm partial sums of the written gradient (see emb_bwd_sq_kernel).
void embedding_bwd_(const at::Tensor& dy, const at::Tensor& tokens, const at::Tensor& dw,
                    bool accumulate, const std::optional<at::Tensor>& part) {
  FT_CHECK_CUDA(dy);
  FT_CHECK_MODEL_DTYPE(dy);
  TORCH_CHECK(dy.scalar_type() == dw.scalar_type(), "embedding_bwd: dtype mismatch");
  FT_CHECK_CONTIG(dy);
  FT_CHECK_CONTIG(dw);
  const int D = dw.size(1);
  const int T = tokens.numel();
  TORCH_CHECK(dy.numel() == (long)T * D, "embedding_bwd: shape mismatch");
  const at::DeviceGuard guard(dw.device());
  TORCH_CHECK(tokens.scalar_type() == at::kLong, "embedding_bwd: tokens must be int64");
  const long V = dw.size(0);
  TORCH_CHECK(V >= 1 && V < (1L << 30), "embedding_bwd: vocabulary size out of range");
  int bits = 1;
  while ((1L << bits) < V) ++bits;
  const int passes = (bits + SORT_BITS - 1) / SORT_BITS;
  auto flat = tokens.reshape({-1}).contiguous();
  if (!accumulate) FT_HIP_CHECK(hipMemsetAsync(dw.data_ptr(), 0, dw.nbytes(), ft_stream()));
  if (T > 0) {
    auto kv = at::empty({4, (long)T}, tokens.options().dtype(at::kInt));  // keys[2][T], vals[2][T]
    int* keys = mptr<int>(kv);
    int* vals = keys + 2L * T;
    hipLaunchKernelGGL(tok_sort_kernel, dim3(1), dim3(SORT_NT), 0, ft_stream(), cptr<int64_t>(flat), T, passes,
                       keys, vals);
    FT_LAUNCH_CHECK();
    const long fin = (long)((passes - 1) & 1) * T;
    const int blocks = (T * 64 + 255) / 256;
    const bool sq = part.has_value() && part->defined();
    if (sq) {
      TORCH_CHECK(!accumulate, "embedding_bwd: norm partials need a fresh gradient");
      FT_CHECK_F32((*part));
      FT_CHECK_CONTIG((*part));
      const int np = (int)part->numel();
      const int g = std::max(1, std::min({blocks, 256, np}));
      FT_DISPATCH_E(dy.scalar_type(),
                    hipLaunchKernelGGL(emb_bwd_sq_kernel<E>, dim3(g), dim3(256), 0, ft_stream(), keys + fin,
                                       vals + fin, cptr<typename E::T>(dy), mptr<typename E::T>(dw), T, D,
                                       mptr<float>(*part), np));
    } else {
      FT_DISPATCH_E(dy.scalar_type(),
                    hipLaunchKernelGGL(emb_bwd_kernel<E>, dim3(blocks), dim3(256), 0, ft_stream(), keys + fin,
                                       vals + fin, cptr<typename E::T>(dy), mptr<typename E::T>(dw), T, D,
                                       accumulate));
    }
  } else if (part.has_value() && part->defined()) {
    part->zero_();
  }
  FT_LAUNCH_CHECK();
}

TORCH_LIBRARY_FRAGMENT(ftamd, m) {
  m.def("embedding_fwd(Tensor tokens, Tensor weight) -> Tensor", &embedding_fwd);
  m.def("embedding_bwd_(Tensor dy, Tensor tokens, Tensor(a!) dw, bool accumulate, Tensor(b!)? part=None) -> ()",
        &embedding_bwd_);
}
