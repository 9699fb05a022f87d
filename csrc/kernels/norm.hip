// RMSNorm / LayerNorm (weight-only) forward + backward for gfx950.
//
// Math parity with the reference RMSNorm (reference model.py:24-48): the
// normalisation runs in fp32, is rounded to the activation dtype, and only then
// multiplied by the weight (`output = norm(x.float()).type_as(x) * weight`).
// `norm_type="layernorm"` (reference model.py:19, declared but unused there)
// selects the mean-subtracting variant.
//
// Layout: one wave (64 lanes) per row, 8 contiguous elements (one 16-B load for
// bf16 / fp16, 32 B for fp32 under --model-dtype) per lane per 512-column chunk;
// the whole row stays in VGPRs between the reduction and the write (one HBM read
// + one write per element). Backward writes per-wave fp32 dW partials (no atomics
// → deterministic) that a column-parallel kernel folds into the weight gradient,
// which is written straight into the flat gradient buffer. Backward grid: ~2 rows per wave so every CU gets
// work (rows are independent; a 64-block grid left 3/4 of the chip idle).
#include "torch_utils.h"

namespace {

constexpr int ROWS_PER_BLOCK = 4;  // 4 waves x 64 lanes

// With ADD: the residual add of the previous sub-block is fused in —
// h1 = x + d (rounded to the model dtype) is written to `hout` (the residual stream) and normalised, so
// the projection GEMMs never need a C input (hipBLASLt copies C into a fresh
// output first) and h1 is read once. Same rounding as the unfused
// `x = x + f(x)` (model-dtype add) followed by the norm.
template <class E, int CH, bool LN, bool ADD>
__global__ __launch_bounds__(256) void norm_fwd_kernel(const typename E::T* __restrict__ x,
                                                       const typename E::T* __restrict__ d,
                                                       typename E::T* __restrict__ hout,
                                                       const typename E::T* __restrict__ w,
                                                       typename E::T* __restrict__ y,
                                                       float* __restrict__ rstd,
                                                       float* __restrict__ mean_out, int M,
                                                       int N, float eps) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * ROWS_PER_BLOCK + (threadIdx.x >> 6);
  if (row >= M) return;
  using T = typename E::T;
  const T* xr = x + (size_t)row * N;
  float v[CH][8];
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < CH; ++c) {
    const int idx = c * 512 + lane * 8;
    if (idx < N) {
      ld8<E>(xr + idx, v[c]);
      if constexpr (ADD) {
        float dv[8];
        ld8<E>(d + (size_t)row * N + idx, dv);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[c][j] = rnd<E>(v[c][j] + dv[j]);
        st8<E>(hout + (size_t)row * N + idx, v[c]);
      }
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[c][j] = 0.f;
    }
    if (LN) {
#pragma unroll
      for (int j = 0; j < 8; ++j) s += v[c][j];
    }
  }
  float mu = 0.f;
  if (LN) mu = wave_sum(s) / (float)N;
  float ss = 0.f;
#pragma unroll
  for (int c = 0; c < CH; ++c) {
    const int idx = c * 512 + lane * 8;
    if (idx < N) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float d = v[c][j] - mu;
        ss += d * d;
      }
    }
  }
  ss = wave_sum(ss);
  const float r = rsqrtf(ss / (float)N + eps);
  T* yr = y + (size_t)row * N;
#pragma unroll
  for (int c = 0; c < CH; ++c) {
    const int idx = c * 512 + lane * 8;
    if (idx < N) {
      float wf[8], o[8];
      ld8<E>(w + idx, wf);
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = rnd<E>((v[c][j] - mu) * r) * wf[j];
      st8<E>(yr + idx, o);
    }
  }
  if (lane == 0) {
    rstd[row] = r;
    if (LN) mean_out[row] = mu;
  }
}

// dx = r * (dn - mean(dn) [LN only] - n * mean(dn * n)),  dn = dy * w, n = (x - mu) * r
// dw_partial[wave_slot][col] += dy * n
template <class E, int CH, bool LN>
__global__ __launch_bounds__(256) void norm_bwd_kernel(
    const typename E::T* __restrict__ dy, const typename E::T* __restrict__ x,
    const typename E::T* __restrict__ w, const float* __restrict__ rstd,
    const float* __restrict__ mean_in, typename E::T* __restrict__ dx,
    const typename E::T* __restrict__ dres, float* __restrict__ dw_part, int M, int N) {
  using T = typename E::T;
  // Row data is kept packed (model dtype) in VGPRs; fp32 values are recomputed per pass
  // to keep the register footprint at ~3 x CH x 4 + 8 x CH VGPRs.
  const int lane = threadIdx.x & 63;
  const int slot = blockIdx.x * ROWS_PER_BLOCK + (threadIdx.x >> 6);
  const int nslots = gridDim.x * ROWS_PER_BLOCK;
  P8<E> wr[CH];  // (N <= 8192: the LDS fold below needs N*4 bytes)
  float acc[CH][8];
  const P8<E> z = zp8<E>();
#pragma unroll
  for (int c = 0; c < CH; ++c) {
    const int idx = c * 512 + lane * 8;
    wr[c] = idx < N ? ldp8<E>(w + idx) : z;
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[c][j] = 0.f;
  }
  const float invN = 1.f / (float)N;
  for (int row = slot; row < M; row += nslots) {
    const float r = rstd[row];
    const float mu = LN ? mean_in[row] : 0.f;
    const T* xr = x + (size_t)row * N;
    const T* dyr = dy + (size_t)row * N;
    const T* drr = dres ? dres + (size_t)row * N : nullptr;
    // all three row loads are issued together (one HBM round trip per row, not two)
    P8<E> xv[CH], gv[CH], rv[CH];
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      const int idx = c * 512 + lane * 8;
      xv[c] = idx < N ? ldp8<E>(xr + idx) : z;
      gv[c] = idx < N ? ldp8<E>(dyr + idx) : z;
      rv[c] = (drr && idx < N) ? ldp8<E>(drr + idx) : z;
    }
    float sdn = 0.f, sdnn = 0.f;
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      float xf[8], g[8], wf[8];
      unp8<E>(xv[c], xf);
      unp8<E>(gv[c], g);
      unp8<E>(wr[c], wf);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float n = (xf[j] - mu) * r;
        const float dn = g[j] * wf[j];
        acc[c][j] += g[j] * n;
        sdn += dn;
        sdnn += dn * n;
      }
    }
    sdnn = wave_sum(sdnn) * invN;
    if (LN) sdn = wave_sum(sdn) * invN;
    T* dxr = dx + (size_t)row * N;
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      const int idx = c * 512 + lane * 8;
      if (idx < N) {
        float xf[8], g[8], wf[8], o[8];
        unp8<E>(xv[c], xf);
        unp8<E>(gv[c], g);
        unp8<E>(wr[c], wf);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float n = (xf[j] - mu) * r;
          o[j] = r * (g[j] * wf[j] - (LN ? sdn : 0.f) - n * sdnn);
        }
        if (drr) {
          float rr[8];
          unp8<E>(rv[c], rr);
#pragma unroll
          for (int j = 0; j < 8; ++j) o[j] += rr[j];
        }
        st8<E>(dxr + idx, o);
      }
    }
  }
  // Fold the 4 waves' dW partials in LDS (fixed wave order: deterministic), then one
  // coalesced fp32 row per block -> the column-sum kernel reads nblk rows, not 4*nblk.
  extern __shared__ __attribute__((aligned(16))) float red[];  // [N]
  const int wave = threadIdx.x >> 6;
#pragma unroll 1
  for (int w = 0; w < ROWS_PER_BLOCK; ++w) {
    if (wave == w) {
#pragma unroll
      for (int c = 0; c < CH; ++c) {
        const int idx = c * 512 + lane * 8;
        if (idx < N) {
          float4* r4 = reinterpret_cast<float4*>(red + idx);
          if (w == 0) {
            r4[0] = make_float4(acc[c][0], acc[c][1], acc[c][2], acc[c][3]);
            r4[1] = make_float4(acc[c][4], acc[c][5], acc[c][6], acc[c][7]);
          } else {
            float4 a = r4[0], b = r4[1];
            a.x += acc[c][0]; a.y += acc[c][1]; a.z += acc[c][2]; a.w += acc[c][3];
            b.x += acc[c][4]; b.y += acc[c][5]; b.z += acc[c][6]; b.w += acc[c][7];
            r4[0] = a;
            r4[1] = b;
          }
        }
      }
    }
    __syncthreads();
  }
  float* part = dw_part + (size_t)blockIdx.x * N;
  for (int i = threadIdx.x * 4; i < N; i += 256 * 4)
    *reinterpret_cast<float4*>(part + i) = *reinterpret_cast<const float4*>(red + i);
}

// Split-row backward: a 1024-thread block = 4 row groups x 4 waves; the 4 waves of a
// group share one row (wave q owns 512-column chunks q, q+4, ...), so a wave holds
// CHW = chunks/4 chunks instead of the whole row. The freed registers buy two rows per
// group in flight (all of a block's 8 rows are requested in one round trip) and 16
// waves per CU instead of 4 — the one-wave-per-row kernel above spends most of its
// time waiting on its single round of loads. Row sums cross waves through LDS
// (double-buffered by iteration parity: one barrier per iteration). dW partials fold
// in LDS in fixed group order -> one fp32 row per block (deterministic), as above.
constexpr int SPLIT = 4;    // waves per row
constexpr int GROUPS = 4;   // row groups per block
constexpr int RPI = 1;      // rows per group per iteration (loads issued together)

template <class E, int CHW, bool LN>
__global__ __launch_bounds__(1024) void norm_bwd_split_kernel(
    const typename E::T* __restrict__ dy, const typename E::T* __restrict__ x,
    const typename E::T* __restrict__ w, const float* __restrict__ rstd,
    const float* __restrict__ mean_in, typename E::T* __restrict__ dx,
    const typename E::T* __restrict__ dres, float* __restrict__ dw_part, int M, int N,
    int rows_per_block) {
  using T = typename E::T;
  __shared__ float sums[2][GROUPS][RPI][2][SPLIT];  // [parity][group][row][sdnn|sdn][wave]
  extern __shared__ __attribute__((aligned(16))) float red[];  // [N]
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int q = wave % SPLIT, grp = wave / SPLIT;
  const int row0 = blockIdx.x * rows_per_block;
  const P8<E> z = zp8<E>();
  P8<E> wr[CHW];
  float acc[CHW][8];
#pragma unroll
  for (int c = 0; c < CHW; ++c) {
    const int idx = (c * SPLIT + q) * 512 + lane * 8;
    wr[c] = idx < N ? ldp8<E>(w + idx) : z;
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[c][j] = 0.f;
  }
  const float invN = 1.f / (float)N;
  const int iters = rows_per_block / (GROUPS * RPI);  // block-uniform trip count (barriers)
  for (int it = 0; it < iters; ++it) {
    const int par = it & 1;
    int rows[RPI];
    P8<E> xv[RPI][CHW], gv[RPI][CHW];
#pragma unroll
    for (int k = 0; k < RPI; ++k) {
      const int rr = row0 + (it * RPI + k) * GROUPS + grp;
      rows[k] = (rr < M && rr < row0 + rows_per_block) ? rr : -1;
      const size_t off = (size_t)(rows[k] < 0 ? 0 : rows[k]) * N;
#pragma unroll
      for (int c = 0; c < CHW; ++c) {
        const int idx = (c * SPLIT + q) * 512 + lane * 8;
        const bool ok = rows[k] >= 0 && idx < N;
        xv[k][c] = ok ? ldp8<E>(x + off + idx) : z;
        gv[k][c] = ok ? ldp8<E>(dy + off + idx) : z;
      }
    }
    float r[RPI], mu[RPI];
#pragma unroll
    for (int k = 0; k < RPI; ++k) {
      r[k] = rows[k] >= 0 ? rstd[rows[k]] : 0.f;
      mu[k] = (LN && rows[k] >= 0) ? mean_in[rows[k]] : 0.f;
      float sdn = 0.f, sdnn = 0.f;
#pragma unroll
      for (int c = 0; c < CHW; ++c) {
        float xf[8], g[8], wf[8];
        unp8<E>(xv[k][c], xf);
        unp8<E>(gv[k][c], g);
        unp8<E>(wr[c], wf);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float n = (xf[j] - mu[k]) * r[k];
          const float dn = g[j] * wf[j];
          acc[c][j] += g[j] * n;
          sdn += dn;
          sdnn += dn * n;
        }
      }
      sdnn = wave_sum(sdnn);
      if (LN) sdn = wave_sum(sdn);
      if (lane == 0) {
        sums[par][grp][k][0][q] = sdnn;
        if (LN) sums[par][grp][k][1][q] = sdn;
      }
    }
    __syncthreads();
    // Opaque to the optimiser: the fp32 unpacks are redone from the packed registers
    // instead of being kept alive across the barrier (which spilled at 128 VGPRs).
#pragma unroll
    for (int k = 0; k < RPI; ++k)
#pragma unroll
      for (int c = 0; c < CHW; ++c) {
        pin8<E>(xv[k][c]);
        pin8<E>(gv[k][c]);
      }
#pragma unroll
    for (int c = 0; c < CHW; ++c) pin8<E>(wr[c]);
#pragma unroll
    for (int k = 0; k < RPI; ++k) {
      if (rows[k] < 0) continue;
      float sdnn = 0.f, sdn = 0.f;
#pragma unroll
      for (int s = 0; s < SPLIT; ++s) {  // fixed order: every wave of the row gets the same sum
        sdnn += sums[par][grp][k][0][s];
        if (LN) sdn += sums[par][grp][k][1][s];
      }
      sdnn *= invN;
      sdn *= invN;
      T* dxr = dx + (size_t)rows[k] * N;
#pragma unroll
      for (int c = 0; c < CHW; ++c) {
        const int idx = (c * SPLIT + q) * 512 + lane * 8;
        if (idx < N) {
          float xf[8], g[8], wf[8], o[8];
          unp8<E>(xv[k][c], xf);
          unp8<E>(gv[k][c], g);
          unp8<E>(wr[c], wf);
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const float n = (xf[j] - mu[k]) * r[k];
            o[j] = r[k] * (g[j] * wf[j] - (LN ? sdn : 0.f) - n * sdnn);
          }
          if (dres) {  // loaded after the barrier: keeps the pre-barrier set at 2 operands
            float rr[8];
            ld8<E>(dres + (size_t)rows[k] * N + idx, rr);
#pragma unroll
            for (int j = 0; j < 8; ++j) o[j] += rr[j];
          }
          st8<E>(dxr + idx, o);
        }
      }
    }
  }
#pragma unroll 1
  for (int g = 0; g < GROUPS; ++g) {
    if (grp == g) {
#pragma unroll
      for (int c = 0; c < CHW; ++c) {
        const int idx = (c * SPLIT + q) * 512 + lane * 8;
        if (idx < N) {
          float4* r4 = reinterpret_cast<float4*>(red + idx);
          if (g == 0) {
            r4[0] = make_float4(acc[c][0], acc[c][1], acc[c][2], acc[c][3]);
            r4[1] = make_float4(acc[c][4], acc[c][5], acc[c][6], acc[c][7]);
          } else {
            float4 a = r4[0], b = r4[1];
            a.x += acc[c][0]; a.y += acc[c][1]; a.z += acc[c][2]; a.w += acc[c][3];
            b.x += acc[c][4]; b.y += acc[c][5]; b.z += acc[c][6]; b.w += acc[c][7];
            r4[0] = a;
            r4[1] = b;
          }
        }
      }
    }
    __syncthreads();
  }
  float* part = dw_part + (size_t)blockIdx.x * N;
  for (int i = threadIdx.x * 4; i < N; i += 1024 * 4)
    *reinterpret_cast<float4*>(part + i) = *reinterpret_cast<const float4*>(red + i);
}

// Column sums of a [P, N] fp32 slab -> model-dtype dw (optionally accumulated).
// Block = 32 columns x 8 row groups (128-B row segments); fixed summation order
// (deterministic). 128 blocks for N = 4096.
// sq (optional): block i writes sq[i] = the sum of squares of its 32 stored dw values (the
// gradient norm's partials, ops/grad_sink.py: no separate pass over the norm weights' gradient).
template <class E>
__global__ __launch_bounds__(256) void colsum_kernel(const float* __restrict__ part,
                                                     typename E::T* __restrict__ dw, int P, int N,
                                                     bool accumulate, float* __restrict__ sq) {
  __shared__ float red[8][33];
  const int cl = threadIdx.x & 31, g = threadIdx.x >> 5;
  const int col = blockIdx.x * 32 + cl;
  float s = 0.f;
  if (col < N) {
#pragma unroll 4
    for (int p = g; p < P; p += 8) s += part[(size_t)p * N + col];
  }
  red[g][cl] = s;
  __syncthreads();
  if (g == 0) {  // lanes 0..31 of wave 0
    float q = 0.f;
    if (col < N) {
      float t = 0.f;
#pragma unroll
      for (int k = 0; k < 8; ++k) t += red[k][cl];
      if (accumulate) t += ld1<E>(dw + col);
      const typename E::T o = cvt1<E>(t);
      dw[col] = o;
      const float f = ld1<E>(&o);
      q = f * f;
    }
    if (sq != nullptr) {
#pragma unroll
      for (int o = 16; o > 0; o >>= 1) q += __shfl_xor(q, o, 32);
      if (cl == 0) sq[blockIdx.x] = q;
    }
  }
}

template <class E, bool LN, bool ADD>
void launch_fwd(const typename E::T* x, const typename E::T* d, typename E::T* hout,
                const typename E::T* w, typename E::T* y, float* rstd, float* mean, int M, int N,
                float eps, hipStream_t st) {
  const int chunks = (N + 511) / 512;
  dim3 grid((M + ROWS_PER_BLOCK - 1) / ROWS_PER_BLOCK), block(256);
#define FT_NF(C)                                                                             \
  hipLaunchKernelGGL((norm_fwd_kernel<E, C, LN, ADD>), grid, block, 0, st, x, d, hout, w, y, rstd, \
                     mean, M, N, eps)
  if (chunks <= 1) FT_NF(1);
  else if (chunks <= 2) FT_NF(2);
  else if (chunks <= 4) FT_NF(4);
  else if (chunks <= 8) FT_NF(8);
  else if (chunks <= 16) FT_NF(16);
  else TORCH_CHECK(false, "norm: N too large");
#undef FT_NF
}

// Split-row kernel when every wave owns at least one chunk (N >= 2048) and the LDS
// fold fits (N <= 8192); FT_NORM_BWD_SPLIT=0 selects the one-wave-per-row kernel (A/B).
bool use_split_bwd(int N) {
  const char* e = std::getenv("FT_NORM_BWD_SPLIT");
  if (e && e[0] == '0') return false;
  const int chunks = (N + 511) / 512;
  return chunks >= SPLIT && chunks <= 2 * SPLIT;  // CHW <= 2: no spills at 4 waves/SIMD
}

// rows per block: a multiple of GROUPS*RPI, at most one block per CU
void split_grid(int M, int* nblk, int* rows_per_block) {
  const int unit = GROUPS * RPI;
  int nb = std::max(1, std::min(256, (M + unit - 1) / unit));
  int rpb = ((M + nb - 1) / nb + unit - 1) / unit * unit;
  *rows_per_block = rpb;
  *nblk = std::max(1, (M + rpb - 1) / rpb);
}

template <class E, bool LN>
void launch_bwd_split(const typename E::T* dy, const typename E::T* x, const typename E::T* w,
                      const float* rstd, const float* mean, typename E::T* dx,
                      const typename E::T* dres, float* part, int nblk, int rows_per_block, int M,
                      int N, hipStream_t st) {
  const int chw = ((N + 511) / 512 + SPLIT - 1) / SPLIT;
  dim3 grid(nblk), block(1024);
  const size_t lds = (size_t)N * sizeof(float);
#define FT_NBS(C)                                                                       \
  hipLaunchKernelGGL((norm_bwd_split_kernel<E, C, LN>), grid, block, lds, st, dy, x, w, rstd, \
                     mean, dx, dres, part, M, N, rows_per_block)
  if (chw <= 1) FT_NBS(1);
  else if (chw <= 2) FT_NBS(2);
  else if (chw <= 4) FT_NBS(4);
  else TORCH_CHECK(false, "norm: N too large for the split kernel");
#undef FT_NBS
}

template <class E, bool LN>
void launch_bwd(const typename E::T* dy, const typename E::T* x, const typename E::T* w,
                const float* rstd, const float* mean, typename E::T* dx, const typename E::T* dres,
                float* part, int nblk, int M, int N, hipStream_t st) {
  const int chunks = (N + 511) / 512;
  dim3 grid(nblk), block(256);
  const size_t lds = (size_t)N * sizeof(float);
#define FT_NB(C)                                                                            \
  hipLaunchKernelGGL((norm_bwd_kernel<E, C, LN>), grid, block, lds, st, dy, x, w, rstd, mean, dx, \
                     dres, part, M, N)
  if (chunks <= 1) FT_NB(1);
  else if (chunks <= 2) FT_NB(2);
  else if (chunks <= 4) FT_NB(4);
  else if (chunks <= 8) FT_NB(8);
  else if (chunks <= 16) FT_NB(16);
  else TORCH_CHECK(false, "norm: N too large");
#undef FT_NB
}

}  // namespace

// Returns (y, rstd, mean, h). `mean` is empty for RMSNorm. With `d` given, the input
// is h = x + d rounded to the model dtype (fused residual add) and h is returned;
// otherwise h is empty. x, d, w, y, h: bf16 / fp16 / fp32 (one dtype).
std::tuple<at::Tensor, at::Tensor, at::Tensor, at::Tensor> add_norm_fwd(
    const at::Tensor& x, const std::optional<at::Tensor>& d, const at::Tensor& w, double eps,
    bool layernorm) {
  FT_CHECK_CUDA(x);
  FT_CHECK_MODEL_DTYPE(x);
  FT_CHECK_CONTIG(x);
  FT_CHECK_CONTIG(w);
  TORCH_CHECK(w.scalar_type() == x.scalar_type(), "norm: weight dtype must match x");
  const int N = x.size(-1);
  TORCH_CHECK(w.numel() == N, "norm: weight size mismatch");
  TORCH_CHECK(N % 8 == 0, "norm: N must be a multiple of 8");
  const int M = x.numel() / N;
  const bool add = d.has_value() && d->defined();
  if (add) {
    TORCH_CHECK(d->scalar_type() == x.scalar_type(), "add_norm: delta dtype must match x");
    FT_CHECK_CONTIG((*d));
    TORCH_CHECK(d->numel() == x.numel(), "add_norm: residual delta shape mismatch");
  }
  const at::DeviceGuard guard(x.device());
  auto y = at::empty_like(x);
  auto rstd = at::empty({M}, x.options().dtype(at::kFloat));
  at::Tensor mean = at::empty({layernorm ? M : 0}, x.options().dtype(at::kFloat));
  at::Tensor h = add ? at::empty_like(x) : at::empty({0}, x.options());
  if (M == 0) return {y, rstd, mean, h};
  float* mp = layernorm ? mptr<float>(mean) : nullptr;
  FT_DISPATCH_E(x.scalar_type(), {
    using T = typename E::T;
    const T* dp = add ? cptr<T>(*d) : nullptr;
    T* hp = add ? mptr<T>(h) : nullptr;
    auto go = [&](auto ln, auto ad) {
      launch_fwd<E, decltype(ln)::value, decltype(ad)::value>(
          cptr<T>(x), dp, hp, cptr<T>(w), mptr<T>(y), mptr<float>(rstd), mp, M, N, (float)eps,
          ft_stream());
    };
    if (layernorm && add) go(std::true_type{}, std::true_type{});
    else if (layernorm) go(std::true_type{}, std::false_type{});
    else if (add) go(std::false_type{}, std::true_type{});
    else go(std::false_type{}, std::false_type{});
  });
  FT_LAUNCH_CHECK();
  return {y, rstd, mean, h};
}

std::tuple<at::Tensor, at::Tensor, at::Tensor> norm_fwd(const at::Tensor& x, const at::Tensor& w,
                                                       double eps, bool layernorm) {
  auto r = add_norm_fwd(x, std::nullopt, w, eps, layernorm);
  return {std::get<0>(r), std::get<1>(r), std::get<2>(r)};
}

// Returns dx; writes (or accumulates) dw into `dw` (a view into the flat grad buffer).
// `dres` (optional) is added into dx: the residual-stream gradient fused into the norm.
// dx and the per-block fp32 dW partial rows [P, N]; colsum_ folds them into dw. Split so
// the fold can run on the weight-gradient stream (ops/functional.py): during backward the
// compute stream shares the CUs with the dW GEMMs and every small launch on it waits for
// CU slots, so the fold does not belong on the critical path.
std::tuple<at::Tensor, at::Tensor> norm_bwd_part(const at::Tensor& dy, const at::Tensor& x,
                                                 const at::Tensor& w, const at::Tensor& rstd,
                                                 const std::optional<at::Tensor>& mean,
                                                 const std::optional<at::Tensor>& dres) {
  FT_CHECK_CUDA(dy);
  FT_CHECK_CONTIG(dy);
  FT_CHECK_CUDA(x);
  FT_CHECK_MODEL_DTYPE(x);
  FT_CHECK_CONTIG(x);
  FT_CHECK_CONTIG(w);
  TORCH_CHECK(dy.scalar_type() == x.scalar_type() && w.scalar_type() == x.scalar_type(),
              "norm_bwd: dy, x and w must share one dtype");
  FT_CHECK_F32(rstd);
  FT_CHECK_CONTIG(rstd);
  const int N = x.size(-1);
  const int M = x.numel() / N;
  TORCH_CHECK(dy.numel() == x.numel() && w.numel() == N, "norm_bwd: shape mismatch");
  TORCH_CHECK(rstd.numel() == M, "norm_bwd: rstd must hold one value per row");
  TORCH_CHECK(N <= 8192 && N % 8 == 0, "norm_bwd: N must be a multiple of 8 and <= 8192");
  const at::DeviceGuard guard(x.device());
  auto dx = at::empty_like(x);
  const bool ln = mean.has_value() && mean->defined() && mean->numel() > 0;
  const bool has_dres = dres.has_value() && dres->defined();
  if (has_dres) {
    TORCH_CHECK(dres->scalar_type() == x.scalar_type(), "norm_bwd: dres dtype must match x");
    FT_CHECK_CONTIG((*dres));
    TORCH_CHECK(dres->numel() == x.numel(), "norm_bwd: dres shape mismatch");
  }
  // ~2 rows per wave: enough blocks to cover all 256 CUs, few enough partial rows
  int nblk = std::max(1, std::min((M + ROWS_PER_BLOCK * 2 - 1) / (ROWS_PER_BLOCK * 2), 256));
  const bool split = M > 0 && use_split_bwd(N);
  int rows_per_block = 0;
  if (split) split_grid(M, &nblk, &rows_per_block);
  auto part = at::empty({(long)nblk, N}, x.options().dtype(at::kFloat));
  const float* mp = ln ? cptr<float>(*mean) : nullptr;
  if (M > 0) {
    FT_DISPATCH_E(x.scalar_type(), {
      using T = typename E::T;
      const T* dr = has_dres ? cptr<T>(*dres) : nullptr;
      if (split) {
        if (ln)
          launch_bwd_split<E, true>(cptr<T>(dy), cptr<T>(x), cptr<T>(w), cptr<float>(rstd), mp,
                                    mptr<T>(dx), dr, mptr<float>(part), nblk, rows_per_block, M,
                                    N, ft_stream());
        else
          launch_bwd_split<E, false>(cptr<T>(dy), cptr<T>(x), cptr<T>(w), cptr<float>(rstd),
                                     nullptr, mptr<T>(dx), dr, mptr<float>(part), nblk,
                                     rows_per_block, M, N, ft_stream());
      } else {
        if (ln)
          launch_bwd<E, true>(cptr<T>(dy), cptr<T>(x), cptr<T>(w), cptr<float>(rstd), mp,
                              mptr<T>(dx), dr, mptr<float>(part), nblk, M, N, ft_stream());
        else
          launch_bwd<E, false>(cptr<T>(dy), cptr<T>(x), cptr<T>(w), cptr<float>(rstd), nullptr,
                               mptr<T>(dx), dr, mptr<float>(part), nblk, M, N, ft_stream());
      }
    });
    FT_LAUNCH_CHECK();
  }
  return {dx, M > 0 ? part : part.narrow(0, 0, 0)};
}

// dw ([N], model dtype) = column sums of part [P, N] (+ dw when accumulating); fixed order.
// sq: ceil(N / 32) fp32 sums of squares of the stored dw, one per 32 columns (optional).
void colsum_(const at::Tensor& part, const at::Tensor& dw, bool accumulate, const std::optional<at::Tensor>& sq) {
  FT_CHECK_CUDA(part);
  FT_CHECK_CONTIG(part);
  FT_CHECK_MODEL_DTYPE(dw);
  FT_CHECK_CONTIG(dw);
  TORCH_CHECK(part.scalar_type() == at::kFloat && part.dim() == 2 && part.size(1) == dw.numel(),
              "colsum_: part must be fp32 [P, N] with N = dw.numel()");
  const at::DeviceGuard guard(dw.device());
  const int N = dw.numel();
  float* sqp = nullptr;
  if (sq.has_value() && sq->defined()) {
    FT_CHECK_F32((*sq));
    FT_CHECK_CONTIG((*sq));
    TORCH_CHECK(sq->numel() >= (N + 31) / 32, "colsum_: sq needs ceil(N / 32) floats");
    sqp = mptr<float>(*sq);
  }
  FT_DISPATCH_E(dw.scalar_type(),
                hipLaunchKernelGGL((colsum_kernel<E>), dim3((N + 31) / 32), dim3(256), 0,
                                   ft_stream(), cptr<float>(part), mptr<typename E::T>(dw),
                                   (int)part.size(0), N, accumulate, sqp));
  FT_LAUNCH_CHECK();
}

at::Tensor norm_bwd(const at::Tensor& dy, const at::Tensor& x, const at::Tensor& w,
                    const at::Tensor& rstd, const std::optional<at::Tensor>& mean,
                    const at::Tensor& dw, const std::optional<at::Tensor>& dres,
                    bool accumulate, const std::optional<at::Tensor>& sq) {
  TORCH_CHECK(dw.numel() == w.numel(), "norm_bwd: dw shape mismatch");
  auto r = norm_bwd_part(dy, x, w, rstd, mean, dres);
  colsum_(std::get<1>(r), dw, accumulate, sq);
  return std::get<0>(r);
}

TORCH_LIBRARY_FRAGMENT(ftamd, m) {
  m.def("norm_fwd(Tensor x, Tensor w, float eps, bool layernorm) -> (Tensor, Tensor, Tensor)",
        &norm_fwd);
  m.def(
      "add_norm_fwd(Tensor x, Tensor? d, Tensor w, float eps, bool layernorm) -> (Tensor, Tensor, "
      "Tensor, Tensor)",
      &add_norm_fwd);
  m.def(
      "norm_bwd_part(Tensor dy, Tensor x, Tensor w, Tensor rstd, Tensor? mean, Tensor? dres) -> "
      "(Tensor, Tensor)",
      &norm_bwd_part);
  m.def("colsum_(Tensor part, Tensor(a!) dw, bool accumulate, Tensor(b!)? sq=None) -> ()", &colsum_);
  m.def(
      "norm_bwd(Tensor dy, Tensor x, Tensor w, Tensor rstd, Tensor? mean, Tensor(a!) dw, "
      "Tensor? dres, bool accumulate, Tensor(b!)? sq=None) -> Tensor",
      &norm_bwd);
}
