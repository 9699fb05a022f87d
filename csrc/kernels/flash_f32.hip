// Causal GQA attention in fp32 (--model-dtype fp32), forward + deterministic backward, gfx950.
//
// The fp32 counterpart of flash_attn.hip for models trained in fp32 (reference utils.py:14-19,
// train.py:54-59: the whole model, attention included, in the chosen dtype; model.py:212 SDPA).
// Every product runs in fp32 on the vector ALUs — no bf16/tf32 MFMA rounding — so the fp32
// model keeps fp32 semantics end to end; it is a precision mode, not the throughput path.
//
// Same packed layouts and GQA indexing as the MFMA kernels (qk [T, ldqk] with Q at h*D and K at
// (Hq+kvh)*D, V in place in qkv [T, (Hq+2Hkv)*D]); lse is natural-log, [B, Hq, S].
// Thread mapping: 4 lanes per row (query row in the forward / dQ kernels, key row in the dK/dV
// kernel), each lane owning D/4 contiguous columns; row dot products are the 4 lanes' partial
// sums folded with two xor-shuffles. K/V (or Q/dO) tiles of 64 rows stage through LDS and are
// read as broadcast float4s (one row per step for the whole block). Online softmax per 64-key
// tile in the forward; the backward is FA2-style with dQ (query-major) and dK/dV (key-major,
// the GQA group's heads summed in fixed order) in separate kernels: no atomics, bit-reproducible.
#include "torch_utils.h"

#include <cmath>

namespace {

constexpr int TR = 64;   // rows per tile (queries or keys)
constexpr int NT = 256;  // threads per block = TR rows x 4 lanes

__device__ __forceinline__ float quad_sum(float v) {
  v += __shfl_xor(v, 1, 64);
  v += __shfl_xor(v, 2, 64);
  return v;
}

template <int DS>
__device__ __forceinline__ void ld_part(const float* p, float* x) {
#pragma unroll
  for (int c = 0; c < DS / 4; ++c) {
    const float4 v = reinterpret_cast<const float4*>(p)[c];
    x[4 * c] = v.x; x[4 * c + 1] = v.y; x[4 * c + 2] = v.z; x[4 * c + 3] = v.w;
  }
}

template <int DS>
__device__ __forceinline__ void st_part(float* p, const float* x, float s) {
#pragma unroll
  for (int c = 0; c < DS / 4; ++c)
    reinterpret_cast<float4*>(p)[c] =
        make_float4(x[4 * c] * s, x[4 * c + 1] * s, x[4 * c + 2] * s, x[4 * c + 3] * s);
}

template <int DS>
__device__ __forceinline__ float dot_part(const float* a, const float* lds) {
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < DS / 4; ++c) {
    const float4 v = reinterpret_cast<const float4*>(lds)[c];
    s = fmaf(a[4 * c], v.x, s);
    s = fmaf(a[4 * c + 1], v.y, s);
    s = fmaf(a[4 * c + 2], v.z, s);
    s = fmaf(a[4 * c + 3], v.w, s);
  }
  return s;
}

template <int DS>
__device__ __forceinline__ void axpy_part(float* acc, float w, const float* lds) {
#pragma unroll
  for (int c = 0; c < DS / 4; ++c) {
    const float4 v = reinterpret_cast<const float4*>(lds)[c];
    acc[4 * c] = fmaf(w, v.x, acc[4 * c]);
    acc[4 * c + 1] = fmaf(w, v.y, acc[4 * c + 1]);
    acc[4 * c + 2] = fmaf(w, v.z, acc[4 * c + 2]);
    acc[4 * c + 3] = fmaf(w, v.w, acc[4 * c + 3]);
  }
}

// Stage TR rows (row0.., clamped to S-1) of a strided [*, ld] source into an LDS [TR][D] image.
template <int D>
__device__ __forceinline__ void stage(float* img, const float* src, long ld, int row0, int S) {
  for (int i = threadIdx.x; i < TR * D / 4; i += NT) {
    const int r = i / (D / 4), c = i % (D / 4);
    const long row = min(row0 + r, S - 1);
    reinterpret_cast<float4*>(img)[i] = *reinterpret_cast<const float4*>(src + row * ld + c * 4);
  }
}

__device__ __forceinline__ void map_block(int L, int nt, int B, int H, int& t, int& b, int& h) {
  // heaviest causal tiles first: tile index descends with the launch order
  t = nt - 1 - L / (B * H);
  const int rem = L % (B * H);
  b = rem / H;
  h = rem % H;
}

template <int D>
__global__ __launch_bounds__(NT) void attn_f32_fwd_kernel(const float* __restrict__ qk,
                                                          const float* __restrict__ qkv,
                                                          float* __restrict__ out,
                                                          float* __restrict__ lse, int B, int S,
                                                          int Hq, int Hkv, float scale, long ldqk) {
  constexpr int DS = D / 4;
  __shared__ __attribute__((aligned(16))) float ks[TR * D];
  __shared__ __attribute__((aligned(16))) float vs[TR * D];
  int qt, b, h;
  map_block(blockIdx.x, (S + TR - 1) / TR, B, Hq, qt, b, h);
  const int kvh = h / (Hq / Hkv);
  const int r = threadIdx.x >> 2, sub = threadIdx.x & 3;
  const int q = qt * TR + r;
  const long ldv = (long)(Hq + 2 * Hkv) * D, ldo = (long)Hq * D;
  const float* Kg = qk + (long)b * S * ldqk + (long)(Hq + kvh) * D;
  const float* Vg = qkv + (long)b * S * ldv + (long)(Hq + Hkv + kvh) * D;
  float qv[DS], o[DS];
  ld_part<DS>(qk + ((long)b * S + min(q, S - 1)) * ldqk + (long)h * D + sub * DS, qv);
#pragma unroll
  for (int i = 0; i < DS; ++i) o[i] = 0.f;
  float m = -INFINITY, l = 0.f;
  const int kend = min((qt + 1) * TR, S);
  for (int k0 = 0; k0 < kend; k0 += TR) {
    __syncthreads();
    stage<D>(ks, Kg, ldqk, k0, S);
    stage<D>(vs, Vg, ldv, k0, S);
    __syncthreads();
    float s[TR];
    float mx = -INFINITY;
#pragma unroll
    for (int j = 0; j < TR; ++j) {
      float x = quad_sum(dot_part<DS>(qv, ks + j * D + sub * DS)) * scale;
      const int key = k0 + j;
      if (key > q || key >= S) x = -INFINITY;
      s[j] = x;
      mx = fmaxf(mx, x);
    }
    const float mn = fmaxf(m, mx);
    const float alpha = m == -INFINITY ? 0.f : expf(m - mn);
    m = mn;
    l *= alpha;
#pragma unroll
    for (int i = 0; i < DS; ++i) o[i] *= alpha;
#pragma unroll
    for (int j = 0; j < TR; ++j) {
      const float p = s[j] == -INFINITY ? 0.f : expf(s[j] - m);
      l += p;
      axpy_part<DS>(o, p, vs + j * D + sub * DS);
    }
  }
  if (q < S) {
    st_part<DS>(out + ((long)b * S + q) * ldo + (long)h * D + sub * DS, o, 1.f / l);
    if (sub == 0) lse[((long)b * Hq + h) * S + q] = m + logf(l);
  }
}

// delta[b, h, q] = sum_d dO * O
template <int D>
__global__ __launch_bounds__(NT) void attn_f32_delta_kernel(const float* __restrict__ dO,
                                                            const float* __restrict__ O,
                                                            float* __restrict__ delta, int B, int S,
                                                            int Hq) {
  constexpr int DS = D / 4;
  const long row = (blockIdx.x * (long)NT + threadIdx.x) >> 2;  // (token, head)
  const int sub = threadIdx.x & 3;
  const long nrows = (long)B * S * Hq;
  float a[DS];
  float acc = 0.f;
  if (row < nrows) {
    ld_part<DS>(dO + row * D + sub * DS, a);
    acc = dot_part<DS>(a, O + row * D + sub * DS);
  }
  acc = quad_sum(acc);
  if (sub == 0 && row < nrows) {
    const long t = row / Hq;
    const int h = (int)(row % Hq);
    delta[((t / S) * Hq + h) * S + t % S] = acc;
  }
}

// dQ[q] = scale * sum_keys dS[q, key] K[key],  dS = P (dP - delta),  P = exp(s - lse)
template <int D>
__global__ __launch_bounds__(NT) void attn_f32_dq_kernel(
    const float* __restrict__ dO, const float* __restrict__ qk, const float* __restrict__ qkv,
    const float* __restrict__ lse, const float* __restrict__ delta, float* __restrict__ dqkv, int B,
    int S, int Hq, int Hkv, float scale, long ldqk) {
  constexpr int DS = D / 4;
  __shared__ __attribute__((aligned(16))) float ks[TR * D];
  __shared__ __attribute__((aligned(16))) float vs[TR * D];
  int qt, b, h;
  map_block(blockIdx.x, (S + TR - 1) / TR, B, Hq, qt, b, h);
  const int kvh = h / (Hq / Hkv);
  const int r = threadIdx.x >> 2, sub = threadIdx.x & 3;
  const int q = qt * TR + r, qc = min(q, S - 1);
  const long ldv = (long)(Hq + 2 * Hkv) * D, ldo = (long)Hq * D;
  const float* Kg = qk + (long)b * S * ldqk + (long)(Hq + kvh) * D;
  const float* Vg = qkv + (long)b * S * ldv + (long)(Hq + Hkv + kvh) * D;
  float qv[DS], dov[DS], dq[DS];
  ld_part<DS>(qk + ((long)b * S + qc) * ldqk + (long)h * D + sub * DS, qv);
  ld_part<DS>(dO + ((long)b * S + qc) * ldo + (long)h * D + sub * DS, dov);
#pragma unroll
  for (int i = 0; i < DS; ++i) dq[i] = 0.f;
  const float lq = lse[((long)b * Hq + h) * S + qc];
  const float dl = delta[((long)b * Hq + h) * S + qc];
  const int kend = min((qt + 1) * TR, S);
  for (int k0 = 0; k0 < kend; k0 += TR) {
    __syncthreads();
    stage<D>(ks, Kg, ldqk, k0, S);
    stage<D>(vs, Vg, ldv, k0, S);
    __syncthreads();
#pragma unroll 4
    for (int j = 0; j < TR; ++j) {
      const float* kr = ks + j * D + sub * DS;
      const float s = quad_sum(dot_part<DS>(qv, kr)) * scale;
      const float dp = quad_sum(dot_part<DS>(dov, vs + j * D + sub * DS));
      const int key = k0 + j;
      const float p = (key > q || key >= S) ? 0.f : expf(s - lq);
      axpy_part<DS>(dq, p * (dp - dl), kr);
    }
  }
  if (q < S) st_part<DS>(dqkv + ((long)b * S + q) * ldv + (long)h * D + sub * DS, dq, scale);
}

// dK[key] = scale * sum_{h in group, q} dS[q, key] Q[q],  dV[key] = sum_{h in group, q} P[q, key] dO[q]
template <int D>
__global__ __launch_bounds__(NT) void attn_f32_dkdv_kernel(
    const float* __restrict__ dO, const float* __restrict__ qk, const float* __restrict__ qkv,
    const float* __restrict__ lse, const float* __restrict__ delta, float* __restrict__ dqkv, int B,
    int S, int Hq, int Hkv, float scale, long ldqk) {
  constexpr int DS = D / 4;
  __shared__ __attribute__((aligned(16))) float qs[TR * D];
  __shared__ __attribute__((aligned(16))) float ds_[TR * D];
  __shared__ float ls[TR], dls[TR];
  int kt, b, kvh;
  map_block(blockIdx.x, (S + TR - 1) / TR, B, Hkv, kt, b, kvh);
  const int G = Hq / Hkv;
  const int r = threadIdx.x >> 2, sub = threadIdx.x & 3;
  const int key = kt * TR + r, kc = min(key, S - 1);
  const long ldv = (long)(Hq + 2 * Hkv) * D, ldo = (long)Hq * D;
  float kv[DS], vv[DS], dk[DS], dv[DS];
  ld_part<DS>(qk + ((long)b * S + kc) * ldqk + (long)(Hq + kvh) * D + sub * DS, kv);
  ld_part<DS>(qkv + ((long)b * S + kc) * ldv + (long)(Hq + Hkv + kvh) * D + sub * DS, vv);
#pragma unroll
  for (int i = 0; i < DS; ++i) dk[i] = dv[i] = 0.f;
  for (int g = 0; g < G; ++g) {  // fixed order over the GQA group: deterministic
    const int h = kvh * G + g;
    const float* Qg = qk + (long)b * S * ldqk + (long)h * D;
    const float* dOg = dO + (long)b * S * ldo + (long)h * D;
    const float* lg = lse + ((long)b * Hq + h) * S;
    const float* dg = delta + ((long)b * Hq + h) * S;
    for (int q0 = kt * TR; q0 < S; q0 += TR) {
      __syncthreads();
      stage<D>(qs, Qg, ldqk, q0, S);
      stage<D>(ds_, dOg, ldo, q0, S);
      if (threadIdx.x < TR) {
        const int qq = min(q0 + (int)threadIdx.x, S - 1);
        ls[threadIdx.x] = lg[qq];
        dls[threadIdx.x] = dg[qq];
      }
      __syncthreads();
      const int n = min(TR, S - q0);
#pragma unroll 4
      for (int i = 0; i < n; ++i) {
        const float* qr = qs + i * D + sub * DS;
        const float* dr = ds_ + i * D + sub * DS;
        const float s = quad_sum(dot_part<DS>(kv, qr)) * scale;
        const float dp = quad_sum(dot_part<DS>(vv, dr));
        const int q = q0 + i;
        const float p = key > q ? 0.f : expf(s - ls[i]);
        axpy_part<DS>(dv, p, dr);
        axpy_part<DS>(dk, p * (dp - dls[i]), qr);
      }
    }
  }
  if (key < S) {
    float* row = dqkv + ((long)b * S + key) * ldv;
    st_part<DS>(row + (long)(Hq + kvh) * D + sub * DS, dk, scale);
    st_part<DS>(row + (long)(Hq + Hkv + kvh) * D + sub * DS, dv, 1.f);
  }
}

void check_f32(const at::Tensor& qk, const at::Tensor& qkv, int64_t S, int64_t Hq, int64_t Hkv,
               int64_t D) {
  FT_CHECK_CUDA(qk);
  FT_CHECK_F32(qk);
  FT_CHECK_F32(qkv);
  FT_CHECK_CONTIG(qk);
  FT_CHECK_CONTIG(qkv);
  TORCH_CHECK(D == 64 || D == 128, "flash_f32: head_dim must be 64 or 128");
  TORCH_CHECK(Hq % Hkv == 0, "flash_f32: Hq must be a multiple of Hkv");
  TORCH_CHECK(qk.size(-1) == (Hq + Hkv) * D || qk.size(-1) == (Hq + 2 * Hkv) * D, "flash_f32: qk width");
  TORCH_CHECK(qkv.size(-1) == (Hq + 2 * Hkv) * D, "flash_f32: qkv width");
  TORCH_CHECK(qk.size(0) == qkv.size(0) && qk.size(0) % S == 0, "flash_f32: rows");
}

}  // namespace

// Returns (o [T, Hq*D] fp32, lse [B, Hq, S] fp32, natural log).
std::tuple<at::Tensor, at::Tensor> flash_f32_fwd(const at::Tensor& qk, const at::Tensor& qkv,
                                                 int64_t S, int64_t Hq, int64_t Hkv, int64_t D) {
  check_f32(qk, qkv, S, Hq, Hkv, D);
  const int T = qk.size(0), B = T / S;
  const at::DeviceGuard guard(qk.device());
  auto out = at::empty({T, Hq * D}, qk.options());
  auto lse = at::empty({B, Hq, S}, qk.options());
  const float scale = 1.f / std::sqrt((float)D);
  const dim3 grid(((S + TR - 1) / TR) * B * Hq);
  if (T > 0) {
    if (D == 128)
      hipLaunchKernelGGL(attn_f32_fwd_kernel<128>, grid, dim3(NT), 0, ft_stream(), cptr<float>(qk),
                         cptr<float>(qkv), mptr<float>(out), mptr<float>(lse), B, (int)S, (int)Hq,
                         (int)Hkv, scale, (long)qk.size(-1));
    else
      hipLaunchKernelGGL(attn_f32_fwd_kernel<64>, grid, dim3(NT), 0, ft_stream(), cptr<float>(qk),
                         cptr<float>(qkv), mptr<float>(out), mptr<float>(lse), B, (int)S, (int)Hq,
                         (int)Hkv, scale, (long)qk.size(-1));
    FT_LAUNCH_CHECK();
  }
  return {out, lse};
}

// Returns dqkv [T, (Hq+2Hkv)*D] fp32 (dQ / dK in the frame of qk, as flash_bwd).
at::Tensor flash_f32_bwd(const at::Tensor& dout, const at::Tensor& qk, const at::Tensor& qkv,
                         const at::Tensor& out, const at::Tensor& lse, int64_t S, int64_t Hq,
                         int64_t Hkv, int64_t D) {
  check_f32(qk, qkv, S, Hq, Hkv, D);
  FT_CHECK_F32(dout);
  FT_CHECK_F32(out);
  FT_CHECK_CONTIG(dout);
  FT_CHECK_CONTIG(out);
  const int T = qk.size(0), B = T / S;
  TORCH_CHECK(dout.numel() == (long)T * Hq * D && out.numel() == (long)T * Hq * D, "flash_f32_bwd: o shape");
  TORCH_CHECK(lse.numel() == (long)B * Hq * S, "flash_f32_bwd: lse shape");
  const at::DeviceGuard guard(qk.device());
  auto dqkv = at::empty({T, (Hq + 2 * Hkv) * D}, qk.options());
  if (T == 0) return dqkv;
  auto delta = at::empty({B, Hq, S}, qk.options());
  const float scale = 1.f / std::sqrt((float)D);
  const long ldqk = qk.size(-1);
  const int nt = (S + TR - 1) / TR;
  const int pre = (int)(((long)T * Hq * 4 + NT - 1) / NT);
#define FT_F32_BWD(DD)                                                                              \
  hipLaunchKernelGGL(attn_f32_delta_kernel<DD>, dim3(pre), dim3(NT), 0, ft_stream(), cptr<float>(dout), \
                     cptr<float>(out), mptr<float>(delta), B, (int)S, (int)Hq);                      \
  hipLaunchKernelGGL(attn_f32_dq_kernel<DD>, dim3(nt * B * Hq), dim3(NT), 0, ft_stream(),            \
                     cptr<float>(dout), cptr<float>(qk), cptr<float>(qkv), cptr<float>(lse),         \
                     cptr<float>(delta), mptr<float>(dqkv), B, (int)S, (int)Hq, (int)Hkv, scale, ldqk); \
  hipLaunchKernelGGL(attn_f32_dkdv_kernel<DD>, dim3(nt * B * Hkv), dim3(NT), 0, ft_stream(),         \
                     cptr<float>(dout), cptr<float>(qk), cptr<float>(qkv), cptr<float>(lse),         \
                     cptr<float>(delta), mptr<float>(dqkv), B, (int)S, (int)Hq, (int)Hkv, scale, ldqk)
  if (D == 128) {
    FT_F32_BWD(128);
  } else {
    FT_F32_BWD(64);
  }
#undef FT_F32_BWD
  FT_LAUNCH_CHECK();
  return dqkv;
}

TORCH_LIBRARY_FRAGMENT(ftamd, m) {
  m.def("flash_f32_fwd(Tensor qk, Tensor qkv, int S, int Hq, int Hkv, int D) -> (Tensor, Tensor)",
        &flash_f32_fwd);
  m.def(
      "flash_f32_bwd(Tensor dout, Tensor qk, Tensor qkv, Tensor out, Tensor lse, int S, int Hq, "
      "int Hkv, int D) -> Tensor",
      &flash_f32_bwd);
}
