// Causal GQA flash attention, forward + backward, for gfx950 (CDNA4).
//
// Replaces the reference's repeat_kv + transpose + F.scaled_dot_product_attention
// (reference model.py:179-215). Inputs are read in place
// from the packed projections:
//   qk  [T, (Hq+Hkv)*D]   rotated Q and K (written by the RoPE kernel)
//   qkv [T, (Hq+2Hkv)*D]  fused QKV projection; V columns start at (Hq+Hkv)*D
// KV head = h / (Hq/Hkv) is indexed directly: no repeat_kv copy, no transposes.
//
// MFMA formulation (v_mfma_f32_32x32x16_bf16, wave64):
//  forward, per wave 32 query rows, per 64-key tile:
//    S^T = K Q^T   (A = K rows from LDS, B = Q^T held in VGPRs for the whole loop)
//      -> the accumulator has the query on the lane and keys in registers, so the
//         row max / row sum of the online softmax are in-lane + one lane^32 swap;
//    O^T += V^T P^T (A = V^T through ds_read_b64_tr_b16 transposed LDS reads,
//         B = P^T taken straight from the S^T accumulator registers, no LDS trip);
//    the running O^T keeps the query on the lane too, so the rescale by
//    exp(m_old - m_new) is a per-lane scalar multiply.
//  backward (FA2 style), per block 128 keys of one (batch, q-head), 4 waves x 32
//    keys, sweeping 32-row query slices from the causal diagonal:
//    S = Q K^T, dP = dO V^T (A = Q / dO rows from LDS, B = K / V in VGPRs),
//    P = exp2(S*c - lse2), dS = P (dP - delta);
//    dV += P^T dO, dK += dS^T Q (A = P / dS straight from accumulators,
//    B = dO / Q through transposed LDS reads);
//    dQ += dS K over the block's 128 keys (dS staged once through LDS) with fp32
//    atomics; dK/dV per q-head partials are folded over the GQA group and
//    converted to bf16 by a finalize kernel.
// LDS images use an XOR swizzle of 16-B chunks that is conflict-free both for
// ds_read_b128 row reads and for the 4-row ds_read_b64_tr_b16 transposed reads
// (cdna_hip_programming.md T2/T10). Block->tile mapping: heavy causal tiles are
// launched first and the GQA siblings of one KV head share blockIdx % 8 (same
// XCD L2 under round-robin dispatch; a speed choice only).
#include "torch_utils.h"

#include <cstdlib>
#include <map>
#include <mutex>
#include <string>
#include <type_traits>
#include <utility>

namespace {

typedef __attribute__((address_space(3))) bf16x4_t lds_bf16x4_t;
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// Compile-time loop: indices are constants before SROA runs, so register arrays
// indexed inside stay in VGPRs (a pragma-unrolled loop is unrolled too late and
// leaves them in scratch / promoted LDS).
template <typename F, int... I>
__device__ __forceinline__ void static_for_impl(F&& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  static_for_impl(f, std::make_integer_sequence<int, N>{});
}

constexpr float LOG2E_F = 1.4426950408889634f;
constexpr float RESCALE_LOG2 = 8.f;  // forward: deferred-rescale threshold (log2 units)

// Byte offset of 16-B chunk c of row r in a [rows][D] bf16 LDS image: 8-row x 32-column
// (512-B) subtiles, 64-B subtile rows, the chunk's low two bits XORed with row bits 2-3
// (cdna_hip_programming.md T10, image (a)). Conflict-free for the ds_read_b128 row reads
// (16 lanes = 16 rows of one chunk) and for the 4-row ds_read_b64_tr_b16 transposed reads;
// and since the XOR never touches the subtile index, reads of other 32-column blocks or
// 8-row blocks are the same lane address plus an immediate, so the 16 transposed reads of
// a 32x32x16 operand sweep share two address registers (the compiler can then keep reads
// in flight ahead of the MFMAs instead of rematerialising addresses).
template <int D>
__device__ __forceinline__ int lds_off(int r, int c) {
  static_assert(D == 64 || D == 128, "head_dim must be 64 or 128");
  return (r >> 3) * (16 * D) + 512 * (c >> 2) + 64 * (r & 7) + 16 * ((c & 3) ^ ((r >> 2) & 3));
}

// Inverse of lds_off: which (row, chunk) lives at 16-B slot P of the image.
template <int D>
__device__ __forceinline__ void lds_inv(int P, int& r, int& c) {
  const int byte = P * 16;
  const int rb = byte / (16 * D), rem = byte % (16 * D);
  const int sub = rem >> 9, r7 = (rem >> 6) & 7, x = (rem >> 4) & 3;
  r = rb * 8 + r7;
  c = sub * 4 + (x ^ ((r >> 2) & 3));
}

// LDS-DMA (global_load_lds_dwordx4): each lane moves 16 B to lds_base + lane * 16.
__device__ __forceinline__ void glds16(const void* g, char* lds_base) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                   (__attribute__((address_space(3))) void*)lds_base, 16, 0, 0);
}

// Fragment types of the 16-bit model dtypes (bf16 default, fp16 under --model-dtype fp16):
// the same 32x32x16 MFMA shape and ds_read_b64_tr_b16 transposed reads exist for both, so the
// kernels below are written once over E and differ only in these four primitives.
typedef _Float16 f16x8_t __attribute__((ext_vector_type(8)));
typedef _Float16 f16x4_t __attribute__((ext_vector_type(4)));
typedef __fp16 fp16x4_raw_t __attribute__((__vector_size__(4 * sizeof(__fp16))));
typedef __attribute__((address_space(3))) fp16x4_raw_t lds_f16x4_t;

template <class E>
struct FA;
template <>
struct FA<EBF16> {
  typedef bf16x8_t v8;
  typedef bf16x4_t v4;
  typedef __bf16 s;
  __device__ static v4 tr(const char* p) {
    return __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4_t*)(p));
  }
  __device__ static f32x16_t mfma(v8 a, v8 b, f32x16_t c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
  }
};
template <>
struct FA<EF16> {
  typedef f16x8_t v8;
  typedef f16x4_t v4;
  typedef _Float16 s;
  __device__ static v4 tr(const char* p) {
    return __builtin_bit_cast(v4, __builtin_amdgcn_ds_read_tr16_b64_v4f16((lds_f16x4_t*)(p)));
  }
  __device__ static f32x16_t mfma(v8 a, v8 b, f32x16_t c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
  }
};

template <class E, int D>
__device__ __forceinline__ typename FA<E>::v8 ld_row(const char* img, int r, int c) {
  return *reinterpret_cast<const typename FA<E>::v8*>(img + lds_off<D>(r, c));
}

template <class V4>
__device__ __forceinline__ auto cat8(V4 a, V4 b) {
  typedef decltype(a[0]) S_;
  typedef std::remove_cv_t<std::remove_reference_t<S_>> S;
  typedef S V8 __attribute__((ext_vector_type(8)));
  V8 r;
  r[0] = a[0]; r[1] = a[1]; r[2] = a[2]; r[3] = a[3];
  r[4] = b[0]; r[5] = b[1]; r[6] = b[2]; r[7] = b[3];
  return r;
}

// Transposed operand fragment from a swizzled [rows][D] image: lane receives
// column col0 + (lane & 31) of rows row0 + 4*hi + (0..3) (elements 0..3) and
// row0 + 8 + 4*hi + (0..3) (elements 4..7) — the k order of an MFMA operand
// built from a 32x32 accumulator's registers 8s..8s+7.
template <class E, int D>
__device__ __forceinline__ typename FA<E>::v8 tr_frag(const char* img, int row0, int col0, int lane) {
  const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3, hi = lane >> 5;
  const int col = col0 + 16 * (g & 1) + 4 * p;
  const int r = row0 + 4 * hi + q;
  const int sub = ((col >> 2) & 1) * 8;
  const auto a = FA<E>::tr(img + lds_off<D>(r, col >> 3) + sub);
  const auto b = FA<E>::tr(img + lds_off<D>(r + 8, col >> 3) + sub);
  return cat8(a, b);
}

// Same for the unswizzled [keys][32 q] dS image (64-B rows; 4 rows = one bank row).
template <class E>
__device__ __forceinline__ typename FA<E>::v8 tr_frag_ds(const char* img, int row0, int lane) {
  const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3, hi = lane >> 5;
  const int col = 16 * (g & 1) + 4 * p;
  const int r = row0 + 4 * hi + q;
  const auto a = FA<E>::tr(img + r * 64 + col * 2);
  const auto b = FA<E>::tr(img + (r + 8) * 64 + col * 2);
  return cat8(a, b);
}

template <class E, int OFF>
__device__ __forceinline__ typename FA<E>::v8 cvt8(const f32x16_t& v) {
  typedef typename FA<E>::s S;
  typename FA<E>::v8 r;
  r[0] = (S)v[OFF + 0]; r[1] = (S)v[OFF + 1]; r[2] = (S)v[OFF + 2]; r[3] = (S)v[OFF + 3];
  r[4] = (S)v[OFF + 4]; r[5] = (S)v[OFF + 5]; r[6] = (S)v[OFF + 6]; r[7] = (S)v[OFF + 7];
  return r;
}

__device__ __forceinline__ f32x16_t mfma32(bf16x8_t a, bf16x8_t b, f32x16_t c) {
  return FA<EBF16>::mfma(a, b, c);
}
__device__ __forceinline__ f32x16_t mfma32(f16x8_t a, f16x8_t b, f32x16_t c) {
  return FA<EF16>::mfma(a, b, c);
}

// Low 16 bits of `bits` as an E value -> float.
template <class E>
__device__ __forceinline__ float u16f(uint32_t bits) {
  const bf16_t t = (bf16_t)(bits & 0xffffu);
  return ld1<E>(&t);
}

// Raw v_exp_f32 (2^x): exp2f adds denormal range-reduction (cmp + cndmask + ldexp per
// call) that softmax does not need — its arguments are <= 0 and tiny results flush to 0.
__device__ __forceinline__ float fast_exp2(float x) { return __builtin_amdgcn_exp2f(x); }

// max(x[lane], x[lane ^ 32]) with one v_permlane32_swap (no LDS round trip, unlike the
// ds_bpermute behind __shfl_xor): swapping x with itself leaves the low half of the wave
// in one result and the high half in the other, on every lane.
__device__ __forceinline__ float max_lane32(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}

// One output row per lane pair (lanes l and l + 32 hold the same row): lane half hi holds, per
// (db, g), columns db*32 + 8g + 4hi .. +3 (val(db, 4g + j)). Stored as 16-byte pieces: the halves
// swap the 4-column halves the other one completes (one v_permlane32_swap per dword), then each
// lane stores the 8-column chunks of its parity (g even: hi 0, odd: hi 1) — 2 * NDB stores of
// 16 B instead of 4 * NDB of 8 B (the attention epilogue's store tail is issue-bound). Every
// lane must call it (the swaps are wave-wide); `ok` guards the stores only.
template <class E, int NDB, class F>
__device__ __forceinline__ void store_row16(bf16_t* orow, int hi, bool ok, F val) {
#pragma unroll
  for (int db = 0; db < NDB; ++db)
#pragma unroll
    for (int gp = 0; gp < 2; ++gp) {
      const int g0 = 2 * gp, g1 = 2 * gp + 1;
      uint2 pe, po;  // this lane's 4 columns of chunks g0 / g1
      pe.x = pk2<E>(val(db, 4 * g0 + 0), val(db, 4 * g0 + 1));
      pe.y = pk2<E>(val(db, 4 * g0 + 2), val(db, 4 * g0 + 3));
      po.x = pk2<E>(val(db, 4 * g1 + 0), val(db, 4 * g1 + 1));
      po.y = pk2<E>(val(db, 4 * g1 + 2), val(db, 4 * g1 + 3));
      const unsigned sx = hi ? pe.x : po.x, sy = hi ? pe.y : po.y;
      const auto rx = __builtin_amdgcn_permlane32_swap(sx, sx, false, false);  // [0]: low half, [1]: high
      const auto ry = __builtin_amdgcn_permlane32_swap(sy, sy, false, false);
      const unsigned qx = hi ? rx[0] : rx[1], qy = hi ? ry[0] : ry[1];  // the partner's half
      const uint4 o = hi ? make_uint4(qx, qy, po.x, po.y) : make_uint4(pe.x, pe.y, qx, qy);
      if (ok) *reinterpret_cast<uint4*>(orow + db * 32 + 8 * (hi ? g1 : g0)) = o;
    }
}

// lse2 / delta rows are padded to a multiple of 32 queries, so a 32-query slice's
// statistics are whole, aligned float4s (padding entries are never used unmasked).
__host__ __device__ __forceinline__ int stat_stride(int S) { return (S + 31) & ~31; }

__device__ __forceinline__ void map_head(int hh, int Hq, int Hkv, int& h, int& kvh) {
  // hh in [0, Hq) -> (h, kvh) so that the Hq/Hkv siblings of one KV head are
  // Hkv block-ids apart (same XCD when Hkv == 8).
  const int G = Hq / Hkv;
  kvh = hh % Hkv;
  h = kvh * G + hh / Hkv;
}

// ================================================================== forward
// NW = waves per query group (32 queries each). SPLIT = 2 (grids of at most one block per CU:
// B * heads * query tiles <= 256, the GPT-2-sized presets) doubles the block to 2 x NW waves:
// the two halves sweep the even / odd key tiles of the same queries with their own online
// softmax and K/V buffers, and merge (m, l, O) through LDS at the end. That halves the causal
// critical path (the last query tile's sweep over all keys) and gives every SIMD two waves, so
// one's softmax overlaps the other's MFMAs.
template <class E, int D, int NW = 4, int SPLIT = 1>
__global__ __launch_bounds__(64 * NW * SPLIT, 8 / (NW * SPLIT)) void flash_fwd_kernel(
    const bf16_t* __restrict__ qk, const bf16_t* __restrict__ qkv, bf16_t* __restrict__ out,
    float* __restrict__ lse2, int B, int S, int Hq, int Hkv, float sl2, long ldqk_) {
  constexpr int BM = 32 * NW, BN = 64, KS = D / 16, NDB = D / 32;
  constexpr int TILE = BN * D * 2;
  // K | V tiles by LDS-DMA into two separate LDS objects, loop unrolled by two (as in the
  // dQ kernel): no staging VGPRs live across the tile's compute, no drained prefetch.
  __shared__ __attribute__((aligned(16))) char kv0[2 * TILE * SPLIT];
  __shared__ __attribute__((aligned(16))) char kv1[2 * TILE * SPLIT];

  const int nqt = (S + BM - 1) / BM;
  const int per = B * Hq;
  const int L = blockIdx.x;
  // Causal work of q-tile qt is ∝ qt+1. With 2 resident blocks per CU, block L and
  // block L + grid/2 share a CU: the first half runs the heavy tiles heaviest-first,
  // the second half the light tiles lightest-first, so each CU's pair sums to the
  // same work (nqt+1 tiles) instead of heavy+heavy next to light+light.
  int qt;
  if ((nqt & 1) == 0 && L >= (nqt / 2) * per)
    qt = (L - (nqt / 2) * per) / per;
  else
    qt = nqt - 1 - L / per;
  const int rem = L % per;
  const int b = rem / Hq;
  int h, kvh;
  map_head(rem % Hq, Hq, Hkv, h, kvh);

  const int tid = threadIdx.x, lane = tid & 63, l32 = lane & 31, hi = lane >> 5;
  const int half = (tid >> 6) / NW, wave = (tid >> 6) % NW;  // key-tile parity, query group
  const int q0 = qt * BM + wave * 32;
  const int qrow = q0 + l32;
  const long ldqk = ldqk_, ldv = (long)(Hq + 2 * Hkv) * D, ldo = (long)Hq * D;
  const bf16_t* Qg = qk + (long)b * S * ldqk + (long)h * D;
  const bf16_t* Kg = qk + (long)b * S * ldqk + (long)(Hq + kvh) * D;
  const bf16_t* Vg = qkv + (long)b * S * ldv + (long)(Hq + Hkv + kvh) * D;

  typename FA<E>::v8 qf[KS];
  {
    const long qr = min(qrow, S - 1);
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
      qf[ks] = *reinterpret_cast<const typename FA<E>::v8*>(Qg + qr * ldqk + ks * 16 + hi * 8);
  }

  const int kend = min((qt + 1) * BM, S);
  const int ntiles = (kend + BN - 1) / BN;
  constexpr int GPW = TILE / 1024 / NW;  // glds instructions per wave per image
  auto dma = [&](int KT, auto BUF) {
    char* kb_ = (decltype(BUF)::value ? kv1 : kv0) + half * 2 * TILE;
    static_for<GPW>([&](auto I) {
      const int piece = wave * GPW + I;
      int r, c;
      lds_inv<D>(piece * 64 + lane, r, c);
      const long key = min(KT * BN + r, S - 1);
      glds16(Kg + key * ldqk + c * 8, kb_ + piece * 1024);
      glds16(Vg + key * ldv + c * 8, kb_ + TILE + piece * 1024);
    });
  };
  if (half < ntiles) dma(half, std::integral_constant<int, 0>{});

  f32x16_t o[NDB];
#pragma unroll
  for (int db = 0; db < NDB; ++db)
#pragma unroll
    for (int r = 0; r < 16; ++r) o[db][r] = 0.f;
  float m = -INFINITY, l = 0.f;
  // Materialise the Q fragments before the loop: left pending, the compiler's waits for
  // them inside the loop would also drain the next tile's prefetch (in-order vmcnt).
  static_for<KS>([&qf](auto I) { asm volatile("" ::"v"(__builtin_bit_cast(u32x4, qf[I]))); });
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();

  // iteration it: this half's key tile it * SPLIT + half (the halves run the same number of
  // iterations — one may idle in the last — so their barriers pair up)
  auto iter = [&](const int it, auto CUR) {
    constexpr int cur = decltype(CUR)::value;
    const int kt = it * SPLIT + half;
    if (kt + SPLIT < ntiles) dma(kt + SPLIT, std::integral_constant<int, cur ^ 1>{});
    const char* kb = (cur ? kv1 : kv0) + half * 2 * TILE;
    const char* vb = kb + TILE;
    const int k0 = kt * BN;
    const bool v0 = k0 <= q0 + 31;       // wave-uniform: sub-tile 0 has an unmasked key
    const bool v1 = k0 + 32 <= q0 + 31;  // sub-tile 1
    // Two code paths: tiles strictly below the diagonal need no masking at all
    // (most of them), diagonal tiles mask per element. Wave-uniform branch.
    auto tile = [&](auto MASKED) {
      constexpr bool MASK = decltype(MASKED)::value;
      f32x16_t s[2];
#pragma unroll
      for (int j = 0; j < 2; ++j) {
#pragma unroll
        for (int r = 0; r < 16; ++r) s[j][r] = 0.f;
        if (!MASK || j == 0 || v1) {
#pragma unroll
          for (int ks = 0; ks < KS; ++ks)
            s[j] = mfma32(ld_row<E, D>(kb, j * 32 + l32, 2 * ks + hi), qf[ks], s[j]);
        }
      }
      // max over raw scores (the softmax scale is > 0), scale folded into one FMA below
      float mx = -INFINITY;
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          float x = s[j][r];
          if constexpr (MASK) {
            const int key = k0 + j * 32 + (r & 3) + 8 * (r >> 2) + 4 * hi;
            if ((j == 1 && !v1) || key > qrow) x = -INFINITY;
            s[j][r] = x;
          }
          mx = fmaxf(mx, x);
        }
      mx = max_lane32(mx);
      // Deferred rescale (cdna_hip_programming.md T13): the running max only moves when
      // some row of the wave grew by more than RESCALE_LOG2 (in log2 units); otherwise P
      // is exponentiated against the stale max (values up to 2^RESCALE_LOG2, exact in the
      // fp32 accumulators, same relative bf16 rounding) and the O / l rescale is skipped.
      // The decision precedes this tile's exponentials, so nothing is ever half-scaled.
      const float cand = mx * sl2;
      if (__any(cand > m + RESCALE_LOG2)) {
        const float mn = fmaxf(m, cand);
        const float alpha = fast_exp2(m - mn);
        m = mn;
        l *= alpha;
#pragma unroll
        for (int db = 0; db < NDB; ++db)
#pragma unroll
          for (int r = 0; r < 16; ++r) o[db][r] *= alpha;
      }
      float ls = 0.f;
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float p = fast_exp2(fmaf(s[j][r], sl2, -m));
          ls += p;
          s[j][r] = p;
        }
      const typename FA<E>::v8 pb00 = cvt8<E, 0>(s[0]), pb01 = cvt8<E, 8>(s[0]);
      const typename FA<E>::v8 pb10 = cvt8<E, 0>(s[1]), pb11 = cvt8<E, 8>(s[1]);
      l += ls;
#pragma unroll
      for (int db = 0; db < NDB; ++db) {
        o[db] = mfma32(tr_frag<E, D>(vb, 0, db * 32, lane), pb00, o[db]);
        o[db] = mfma32(tr_frag<E, D>(vb, 16, db * 32, lane), pb01, o[db]);
      }
      if (!MASK || v1) {
#pragma unroll
        for (int db = 0; db < NDB; ++db) {
          o[db] = mfma32(tr_frag<E, D>(vb, 32, db * 32, lane), pb10, o[db]);
          o[db] = mfma32(tr_frag<E, D>(vb, 48, db * 32, lane), pb11, o[db]);
        }
      }
    };
    if (v0 && kt < ntiles) {
      if (k0 + BN - 1 > q0)  // some key may exceed some query of this wave
        tile(std::true_type{});
      else
        tile(std::false_type{});
    }
    __builtin_amdgcn_s_waitcnt(0);  // this wave's DMA of its next tile has landed ...
    __syncthreads();                // ... and everyone's; nobody reads this tile any more
  };
  const int nit = (ntiles + SPLIT - 1) / SPLIT;
  for (int it = 0; it < nit; it += 2) {
    iter(it, std::integral_constant<int, 0>{});
    if (it + 1 < nit) iter(it + 1, std::integral_constant<int, 1>{});
  }

  if constexpr (SPLIT == 2) {
    // merge: the odd-tile half parks (m, l, O) in LDS (the K/V buffers are free after the
    // loop's last barrier), the even-tile half rescales both to the common max and adds
    // O in kv0 (NDB * 16 floats per lane), (m, l) in kv1; lane-fastest: conflict-free
    float* xo = reinterpret_cast<float*>(kv0) + (wave * 64 + lane);
    float* xs = reinterpret_cast<float*>(kv1) + (wave * 64 + lane);
    static_assert(NW * 64 * NDB * 16 * 4 <= 2 * TILE * SPLIT, "merge buffer");
    if (half == 1) {
#pragma unroll
      for (int db = 0; db < NDB; ++db)
#pragma unroll
        for (int r = 0; r < 16; ++r) xo[(db * 16 + r) * NW * 64] = o[db][r];
      xs[0] = m;
      xs[NW * 64] = l;
    }
    __syncthreads();
    if (half == 1) return;
    const float m1 = xs[0], l1 = xs[NW * 64];
    const float mn = fmaxf(m, m1);
    // a side that saw no unmasked key keeps m = -inf, l = 0, O = 0: weight 0, never NaN
    const float a0 = m == -INFINITY ? 0.f : fast_exp2(m - mn);
    const float a1 = m1 == -INFINITY ? 0.f : fast_exp2(m1 - mn);
#pragma unroll
    for (int db = 0; db < NDB; ++db)
#pragma unroll
      for (int r = 0; r < 16; ++r) o[db][r] = o[db][r] * a0 + xo[(db * 16 + r) * NW * 64] * a1;
    l = l * a0 + l1 * a1;
    m = mn;
  }

  l += __shfl_xor(l, 32, 64);
  const float inv = 1.f / l;
  store_row16<E, NDB>(out + ((long)b * S + min(qrow, S - 1)) * ldo + (long)h * D, hi, qrow < S,
                      [&](int db, int i) { return o[db][i] * inv; });
  if (qrow < S && hi == 0) lse2[((long)b * Hq + h) * stat_stride(S) + qrow] = m + log2f(l);
}

// ================================================================== forward, software-pipelined
// flash_fwd_kernel<E, D, NW, 1> with the scores of key tile j+1 (S^T = K Q^T, 16 MFMAs) issued
// in the same basic block as tile j's softmax (exp2 / row sum / bf16 packing) and O^T += V^T P^T:
// the MFMAs of one tile run while the VALU of the previous one issues (intra-wave pipelining, the
// FA3 "ping-pong inside a warpgroup"), where the unpipelined loop serialises S -> softmax -> PV
// within the wave and leaves only the co-resident block's wave to fill the gaps.
// The row max of tile j+1 and the deferred-rescale decision close iteration j (in the shadow of
// its PV MFMAs), so iteration j+1's exponentials already see the right running max.
// K and V sit in four LDS objects with different phases: iteration j (phase P = j & 1) reads
// K(j+1) from kb[P^1] and V(j) from vb[P] while K(j+2) streams into kb[P] and V(j+1) into vb[P^1]
// (same 64 KiB per block as the unpipelined kernel; no access names a buffer in flight).
template <class E, int D, int NW = 4>
__global__ __launch_bounds__(64 * NW, 8 / NW) void flash_fwd_pipe_kernel(
    const bf16_t* __restrict__ qk, const bf16_t* __restrict__ qkv, bf16_t* __restrict__ out,
    float* __restrict__ lse2, int B, int S, int Hq, int Hkv, float sl2, long ldqk_,
    long long* __restrict__ prof) {
  constexpr int BM = 32 * NW, BN = 64, KS = D / 16, NDB = D / 32;
  constexpr int TILE = BN * D * 2;
  // timing probe (flash_set_fwd_prof; scripts/flash_fwd_timeline.py): 100 MHz wall clock at
  // entry / after the prologue / after the key loop / after the stores, and the CU the block ran on
  long long pt0 = 0, pt1 = 0, pt2 = 0;
  if (prof) pt0 = __builtin_amdgcn_s_memrealtime();
  __shared__ __attribute__((aligned(16))) char kb0[TILE];
  __shared__ __attribute__((aligned(16))) char kb1[TILE];
  __shared__ __attribute__((aligned(16))) char vb0[TILE];
  __shared__ __attribute__((aligned(16))) char vb1[TILE];
  typedef typename FA<E>::v8 v8;

  const int nqt = (S + BM - 1) / BM;
  const int per = B * Hq;
  const int L = blockIdx.x;
  int qt;  // heavy / light pairing of the resident blocks, as flash_fwd_kernel
  if ((nqt & 1) == 0 && L >= (nqt / 2) * per)
    qt = (L - (nqt / 2) * per) / per;
  else
    qt = nqt - 1 - L / per;
  const int rem = L % per;
  const int b = rem / Hq;
  int h, kvh;
  map_head(rem % Hq, Hq, Hkv, h, kvh);

  const int tid = threadIdx.x, lane = tid & 63, l32 = lane & 31, hi = lane >> 5;
  const int wave = tid >> 6;
  const int q0 = qt * BM + wave * 32;
  const int qrow = q0 + l32;
  const long ldqk = ldqk_, ldv = (long)(Hq + 2 * Hkv) * D, ldo = (long)Hq * D;
  const bf16_t* Qg = qk + (long)b * S * ldqk + (long)h * D;
  const bf16_t* Kg = qk + (long)b * S * ldqk + (long)(Hq + kvh) * D;
  const bf16_t* Vg = qkv + (long)b * S * ldv + (long)(Hq + Hkv + kvh) * D;

  v8 qf[KS];
  {
    const long qr = min(qrow, S - 1);
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
      qf[ks] = *reinterpret_cast<const v8*>(Qg + qr * ldqk + ks * 16 + hi * 8);
  }

  const int kend = min((qt + 1) * BM, S);
  const int ntiles = (kend + BN - 1) / BN;
  // the wave's last key tile with an unmasked key (keys <= q0 + 31, < S); < ntiles
  const int wlast = min(q0 + 31, S - 1) / BN;
  constexpr int GPW = TILE / 1024 / NW;  // LDS-DMA instructions per wave per image
  auto dma = [&](const bf16_t* G, long ld, int KT, char* dst) {
    static_for<GPW>([&](auto I) {
      const int piece = wave * GPW + I;
      int r, c;
      lds_inv<D>(piece * 64 + lane, r, c);
      const long key = min(KT * BN + r, S - 1);
      glds16(G + key * ld + c * 8, dst + piece * 1024);
    });
  };

  f32x16_t o[NDB];
#pragma unroll
  for (int db = 0; db < NDB; ++db)
#pragma unroll
    for (int r = 0; r < 16; ++r) o[db][r] = 0.f;
  float m = -INFINITY, l = 0.f;

  // S^T of key tile kt (sub-tile 1 skipped when it is wholly above this wave's diagonal)
  auto scores = [&](const char* kb, int kt, f32x16_t (&s)[2], auto MASKED) {
    constexpr bool MASK = decltype(MASKED)::value;
    const bool v1 = kt * BN + 32 <= q0 + 31;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
#pragma unroll
      for (int r = 0; r < 16; ++r) s[j][r] = 0.f;
      if (!MASK || j == 0 || v1) {
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) s[j] = mfma32(ld_row<E, D>(kb, j * 32 + l32, 2 * ks + hi), qf[ks], s[j]);
      }
    }
  };
  // causal mask (diagonal tiles) + row max of the raw scores, both halves of the wave
  auto rowmax = [&](f32x16_t (&s)[2], int kt, auto MASKED) {
    constexpr bool MASK = decltype(MASKED)::value;
    const int k0 = kt * BN;
    const bool v1 = k0 + 32 <= q0 + 31;
    float mx = -INFINITY;
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        float x = s[j][r];
        if constexpr (MASK) {
          const int key = k0 + j * 32 + (r & 3) + 8 * (r >> 2) + 4 * hi;
          if ((j == 1 && !v1) || key > qrow) x = -INFINITY;
          s[j][r] = x;
        }
        mx = fmaxf(mx, x);
      }
    return max_lane32(mx);
  };
  // deferred rescale (see flash_fwd_kernel): decided before the tile's exponentials
  auto rescale = [&](float mx) {
    const float cand = mx * sl2;
    if (__any(cand > m + RESCALE_LOG2)) {
      const float mn = fmaxf(m, cand);
      const float alpha = fast_exp2(m - mn);
      m = mn;
      l *= alpha;
#pragma unroll
      for (int db = 0; db < NDB; ++db)
#pragma unroll
        for (int r = 0; r < 16; ++r) o[db][r] *= alpha;
    }
  };
  // P = exp2(s * c - m) as bf16 fragments, row sum into l
  auto probs = [&](f32x16_t (&s)[2], v8 (&pb)[4]) {
    float ls = 0.f;
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float p = fast_exp2(fmaf(s[j][r], sl2, -m));
        ls += p;
        s[j][r] = p;
      }
    pb[0] = cvt8<E, 0>(s[0]);
    pb[1] = cvt8<E, 8>(s[0]);
    pb[2] = cvt8<E, 0>(s[1]);
    pb[3] = cvt8<E, 8>(s[1]);
    l += ls;
  };
  auto pv = [&](const char* vb, const v8 (&pb)[4], bool both) {
#pragma unroll
    for (int db = 0; db < NDB; ++db) {
      o[db] = mfma32(tr_frag<E, D>(vb, 0, db * 32, lane), pb[0], o[db]);
      o[db] = mfma32(tr_frag<E, D>(vb, 16, db * 32, lane), pb[1], o[db]);
    }
    if (both) {
#pragma unroll
      for (int db = 0; db < NDB; ++db) {
        o[db] = mfma32(tr_frag<E, D>(vb, 32, db * 32, lane), pb[2], o[db]);
        o[db] = mfma32(tr_frag<E, D>(vb, 48, db * 32, lane), pb[3], o[db]);
      }
    }
  };

  // prologue: K(0), V(0), K(1) in flight; tile 0's scores, row max and running max
  dma(Kg, ldqk, 0, kb0);
  dma(Vg, ldv, 0, vb0);
  if (ntiles > 1) dma(Kg, ldqk, 1, kb1);
  static_for<KS>([&qf](auto I) { asm volatile("" ::"v"(__builtin_bit_cast(u32x4, qf[I]))); });
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  f32x16_t sa[2], sb[2];
  if (BN - 1 > q0) {
    scores(kb0, 0, sa, std::true_type{});
    rescale(rowmax(sa, 0, std::true_type{}));
  } else {
    scores(kb0, 0, sa, std::false_type{});
    rescale(rowmax(sa, 0, std::false_type{}));
  }
  __syncthreads();  // K(0) read by every wave before K(2) lands in kb0
  if (prof) pt1 = __builtin_amdgcn_s_memrealtime();

  // iteration j, phase P = j & 1: scores of tile j are in (P ? sb : sa), the next tile's go to
  // the other array (static renaming: the loop is unrolled by two)
  auto iter = [&](const int j, auto PH) {
    constexpr int P = decltype(PH)::value;
    char* kfill = P ? kb1 : kb0;        // K(j) consumed -> K(j + 2)
    const char* knext = P ? kb0 : kb1;  // K(j + 1)
    const char* vcur = P ? vb1 : vb0;   // V(j)
    char* vfill = P ? vb0 : vb1;        // V(j - 1) consumed -> V(j + 1)
    f32x16_t(&sc)[2] = P ? sb : sa;
    f32x16_t(&sn)[2] = P ? sa : sb;
    if (j + 2 < ntiles) dma(Kg, ldqk, j + 2, kfill);
    if (j + 1 < ntiles) dma(Vg, ldv, j + 1, vfill);
    if ((j + 2) * BN - 1 <= q0) {
      // steady state: tiles j and j + 1 wholly below this wave's diagonal — one basic block
      v8 pb[4];
      scores(knext, j + 1, sn, std::false_type{});
      probs(sc, pb);
      pv(vcur, pb, true);
      rescale(rowmax(sn, j + 1, std::false_type{}));
    } else if (j <= wlast) {
      const bool nxt = j + 1 <= wlast;
      const bool mask_n = (j + 2) * BN - 1 > q0;
      if (nxt) {
        if (mask_n) scores(knext, j + 1, sn, std::true_type{});
        else scores(knext, j + 1, sn, std::false_type{});
      }
      v8 pb[4];
      probs(sc, pb);
      pv(vcur, pb, j * BN + 32 <= q0 + 31);
      if (nxt) {
        if (mask_n) rescale(rowmax(sn, j + 1, std::true_type{}));
        else rescale(rowmax(sn, j + 1, std::false_type{}));
      }
    }
    __builtin_amdgcn_s_waitcnt(0);  // this wave's DMAs landed ...
    __syncthreads();                // ... and everyone's; K(j + 1) / V(j) are read
  };
  for (int j = 0; j < ntiles; j += 2) {
    iter(j, std::integral_constant<int, 0>{});
    if (j + 1 < ntiles) iter(j + 1, std::integral_constant<int, 1>{});
  }
  if (prof) pt2 = __builtin_amdgcn_s_memrealtime();

  l += __shfl_xor(l, 32, 64);
  const float inv = 1.f / l;
  store_row16<E, NDB>(out + ((long)b * S + min(qrow, S - 1)) * ldo + (long)h * D, hi, qrow < S,
                      [&](int db, int i) { return o[db][i] * inv; });
  if (qrow < S && hi == 0) lse2[((long)b * Hq + h) * stat_stride(S) + qrow] = m + log2f(l);
  if (prof) {
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    if (tid == 0) {
      unsigned hw, xcc;
      asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
      asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
      long long* r = prof + (long)blockIdx.x * 8;
      r[0] = pt0;
      r[1] = pt1;
      r[2] = pt2;
      r[3] = __builtin_amdgcn_s_memrealtime();
      r[4] = hw;
      r[5] = xcc;
      r[6] = qt * 4;
      r[7] = ntiles;
    }
  }
}

// ================================================================== backward
// delta[b,h,q] = sum_d dO * O   (one 16-lane group per (q, h) row, 8 bf16 per lane step)
template <class E, int D>
__global__ __launch_bounds__(256) void flash_bwd_pre_kernel(const bf16_t* __restrict__ dO,
                                                            const bf16_t* __restrict__ O,
                                                            float* __restrict__ delta, int B,
                                                            int S, int Hq) {
  const long row = (blockIdx.x * 256L + threadIdx.x) >> 4;  // (token, head) pair
  const int sub = threadIdx.x & 15;
  const long nrows = (long)B * S * Hq;
  float acc = 0.f;
  if (row < nrows) {
    const bf16_t* a = dO + row * D;
    const bf16_t* c = O + row * D;
    for (int d = sub * 8; d < D; d += 128) {
      float x[8], y[8];
      ld8<E>(a + d, x);
      ld8<E>(c + d, y);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc += x[j] * y[j];
    }
  }
#pragma unroll
  for (int o = 8; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
  if (sub == 0 && row < nrows) {
    const long t = row / Hq;  // token = b*S + q
    const int h = (int)(row % Hq);
    const long bb = t / S, q = t % S;
    delta[(bb * Hq + h) * stat_stride(S) + q] = acc;
  }
}

// DQ: 0 = dQ by fp32 atomics (default), 1 = no dQ stage (dK/dV only; a separate
// deterministic dQ kernel follows), 2 = timing experiment: plain (racy) stores.
template <class E, int D, int DQ = 0>
__global__ __launch_bounds__(256, 1) void flash_bwd_kernel(
    const bf16_t* __restrict__ dO, const bf16_t* __restrict__ qk, const bf16_t* __restrict__ qkv,
    const float* __restrict__ lse2, const float* __restrict__ delta, float* __restrict__ dq_acc,
    bf16_t* __restrict__ dk_part, bf16_t* __restrict__ dv_part, int B, int S, int Hq, int Hkv,
    float sl2, float scale, long ldqk_) {
  constexpr int BK = 128, BQ = 32, KS = D / 16, NDB = D / 32, DCH = D / 8;
  constexpr int KIMG = BK * D * 2;   // K image (keys x D)
  constexpr int QIMG = BQ * D * 2;   // one Q or dO slice
  constexpr int DSIMG = BK * BQ * 2; // dS image [keys][32 q]
  // The two Q|dO slice buffers are separate LDS objects and the slice loop is unrolled
  // by two, so every LDS read names a buffer the in-flight DMA provably does not write:
  // the compiler then does not drain the prefetch (vmcnt(0)) before reading a slice.
  __shared__ __attribute__((aligned(16))) char kds[KIMG + DSIMG];
  __shared__ __attribute__((aligned(16))) char qdb0[2 * QIMG];  // [Q | dO], buffer 0
  __shared__ __attribute__((aligned(16))) char qdb1[2 * QIMG];  // [Q | dO], buffer 1
  char* kimg = kds;
  char* dsimg = kds + KIMG;

  const int per = B * Hq;
  const int L = blockIdx.x;
  const int kt = L / per;  // key tile; kt = 0 has the most query slices -> launched first
  const int rem = L % per;
  const int b = rem / Hq;
  int h, kvh;
  map_head(rem % Hq, Hq, Hkv, h, kvh);

  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, l32 = lane & 31, hi = lane >> 5;
  const int kb0 = kt * BK;
  const int kw = kb0 + wave * 32;  // this wave's first key
  const long ldqk = ldqk_, ldv = (long)(Hq + 2 * Hkv) * D, ldo = (long)Hq * D;
  const bf16_t* Qg = qk + (long)b * S * ldqk + (long)h * D;
  const bf16_t* Kg = qk + (long)b * S * ldqk + (long)(Hq + kvh) * D;
  const bf16_t* Vg = qkv + (long)b * S * ldv + (long)(Hq + Hkv + kvh) * D;
  const bf16_t* dOg = dO + (long)b * S * ldo + (long)h * D;
  const float* lseg = lse2 + ((long)b * Hq + h) * stat_stride(S);
  const float* delg = delta + ((long)b * Hq + h) * stat_stride(S);

  // K and V fragments of this wave's 32 keys -> VGPRs (the S = Q K^T and dP = dO V^T
  // B operands, reused by every query slice); the in-kernel dQ stage (DQ != 1) also
  // needs all 128 keys of K as an LDS image.
  if constexpr (DQ != 1) {
#pragma unroll
    for (int i = 0; i < BK * DCH / 256; ++i) {
      const int id = tid + i * 256, row = id / DCH, c = id % DCH;
      const long key = min(kb0 + row, S - 1);
      *reinterpret_cast<uint4*>(kimg + lds_off<D>(row, c)) =
          *reinterpret_cast<const uint4*>(Kg + key * ldqk + c * 8);
    }
  }
  typename FA<E>::v8 vf[KS], kf[KS];
  {
    const long key = min(kw + l32, S - 1);
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      vf[ks] = *reinterpret_cast<const typename FA<E>::v8*>(Vg + key * ldv + ks * 16 + hi * 8);
      kf[ks] = *reinterpret_cast<const typename FA<E>::v8*>(Kg + key * ldqk + ks * 16 + hi * 8);
    }
  }

  const int qs0 = kb0 / BQ;
  const int nqs = (S + BQ - 1) / BQ;
  // Q / dO slices go global -> LDS by LDS-DMA: the swizzle is applied to the
  // per-lane SOURCE address (the LDS side is lane-linear), no staging VGPRs.
  // The slice's lse / delta (query rows 8g + 4hi + 0..3 of the C layout) go straight
  // to registers, one slice ahead: plain loads whose first use is behind the
  // iteration's closing barrier (an LDS copy of them would make the compiler drain
  // the in-flight DMA before reading it).
  constexpr int GPW = QIMG / 1024 / 4;  // glds instructions per wave per image
  float4 lsn[4], dln[4];
#define BWD_GLDS(QS, BUF)                                                      \
  {                                                                            \
    static_for<GPW>([&](auto I) {                                              \
      const int piece = wave * GPW + I;                                        \
      int r, c;                                                                \
      lds_inv<D>(piece * 64 + lane, r, c);                                     \
      const long q = min((QS) * BQ + r, S - 1);                                \
      char* qd_ = (BUF) ? qdb1 : qdb0;                                         \
      glds16(Qg + q * ldqk + c * 8, qd_ + piece * 1024);                       \
      glds16(dOg + q * ldo + c * 8, qd_ + QIMG + piece * 1024);                \
    });                                                                        \
    static_for<4>([&](auto G) {                                                \
      const int q = (QS) * BQ + 8 * G + 4 * hi;                                \
      lsn[G] = *reinterpret_cast<const float4*>(lseg + q);                     \
      dln[G] = *reinterpret_cast<const float4*>(delg + q);                     \
    });                                                                        \
  }

  BWD_GLDS(qs0, 0)
  __syncthreads();

  f32x16_t dk[NDB], dv[NDB];
#pragma unroll
  for (int db = 0; db < NDB; ++db)
#pragma unroll
    for (int r = 0; r < 16; ++r) dk[db][r] = dv[db][r] = 0.f;

  constexpr int WPD = 4 / NDB;        // waves per d-block in the dQ stage
  constexpr int KPW = BK / WPD;       // keys per wave in the dQ stage
  const int qdb = wave % NDB, qkp = wave / NDB;
  const int key = kw + l32;

  auto iter = [&](const int qs, auto CUR) {
    constexpr int cur = decltype(CUR)::value;
    const bool more = qs + 1 < nqs;
    // Prefetch the next slice into the other buffer before computing this one (its
    // last readers finished behind the previous iteration's closing barrier), so the
    // DMA's latency hides under this slice's MFMAs instead of stalling the barrier.
    float4 lsc[4], dlc[4];
    static_for<4>([&](auto G) {
      lsc[G] = lsn[G];
      dlc[G] = dln[G];
    });
    if (more) BWD_GLDS(qs + 1, cur ^ 1)
    const char* qi = cur ? qdb1 : qdb0;
    const char* di = qi + QIMG;
    const int qb = qs * BQ;
    const bool active = qb + BQ - 1 >= kw;  // wave-uniform
    auto slice = [&](auto MASKED) {
      constexpr bool MASK = decltype(MASKED)::value;
      f32x16_t s, dp;
#pragma unroll
      for (int r = 0; r < 16; ++r) s[r] = dp[r] = 0.f;
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        s = mfma32(ld_row<E, D>(qi, l32, 2 * ks + hi), kf[ks], s);
        dp = mfma32(ld_row<E, D>(di, l32, 2 * ks + hi), vf[ks], dp);
      }
      // C layout: lane -> key (col), registers -> query rows
      static_for<4>([&](auto G) {
        constexpr int g = G;
        const float lv[4] = {lsc[g].x, lsc[g].y, lsc[g].z, lsc[g].w};
        const float dv4[4] = {dlc[g].x, dlc[g].y, dlc[g].z, dlc[g].w};
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const int r = 4 * g + t;
          float p = fast_exp2(fmaf(s[r], sl2, -lv[t]));
          float ds = p * (dp[r] - dv4[t]);
          if constexpr (MASK) {
            // also covers padded rows q >= S, whose lse / delta are uninitialised
            const int q = qb + 8 * g + 4 * hi + t;
            const bool off = key > q || q >= S;
            p = off ? 0.f : p;
            ds = off ? 0.f : ds;
          }
          dp[r] = ds;
          s[r] = p;
        }
      });
      const typename FA<E>::v8 pa[2] = {cvt8<E, 0>(s), cvt8<E, 8>(s)};
      const typename FA<E>::v8 da[2] = {cvt8<E, 0>(dp), cvt8<E, 8>(dp)};
#pragma unroll
      for (int ss = 0; ss < 2; ++ss)
#pragma unroll
        for (int db = 0; db < NDB; ++db) {
          dv[db] = mfma32(pa[ss], tr_frag<E, D>(di, 16 * ss, db * 32, lane), dv[db]);
          dk[db] = mfma32(da[ss], tr_frag<E, D>(qi, 16 * ss, db * 32, lane), dk[db]);
        }
      if constexpr (DQ != 1) {
        // dS -> LDS image [key][q] (4 x 8-B writes per lane) for the in-kernel dQ stage
        char* row = dsimg + (wave * 32 + l32) * 64;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          uint2 v;
          v.x = pk2<E>(dp[4 * g + 0], dp[4 * g + 1]);
          v.y = pk2<E>(dp[4 * g + 2], dp[4 * g + 3]);
          *reinterpret_cast<uint2*>(row + (8 * g + 4 * hi) * 2) = v;
        }
      }
    };
    if (active) {
      // the slice straddles this wave's keys (or the ragged end): mask per element
      if (kw + 31 > qb || qb + BQ > S)
        slice(std::true_type{});
      else
        slice(std::false_type{});
    } else if constexpr (DQ != 1) {
      char* row = dsimg + (wave * 32 + l32) * 64;
#pragma unroll
      for (int g = 0; g < 4; ++g) *reinterpret_cast<uint2*>(row + (8 * g + 4 * hi) * 2) = make_uint2(0, 0);
    }
    // dQ[q, d] += scale * sum_keys dS[q, key] K[key, d]
    if constexpr (DQ != 1) {
      __syncthreads();
      f32x16_t acc;
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[r] = 0.f;
      const int kbeg = qkp * KPW;
      // skip key ranges that are entirely above the causal diagonal for this slice
      if (kb0 + kbeg <= qb + BQ - 1) {
#pragma unroll
        for (int k2 = 0; k2 < KPW / 16; ++k2) {
          const int kk = kbeg + 16 * k2;
          acc = mfma32(tr_frag_ds<E>(dsimg, kk, lane), tr_frag<E, D>(kimg, kk, qdb * 32, lane), acc);
        }
        const int d = qdb * 32 + l32;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int q = qb + (r & 3) + 8 * (r >> 2) + 4 * hi;
          if constexpr (DQ == 0) {
            if (q < S) atomicAdd(dq_acc + ((long)b * S + q) * ldo + (long)h * D + d, acc[r] * scale);
          } else {
            if (q < S) dq_acc[((long)b * S + q) * ldo + (long)h * D + d] = acc[r] * scale;
          }
        }
      }
    }
    __syncthreads();
  };
  for (int qs = qs0; qs < nqs; qs += 2) {
    iter(qs, std::integral_constant<int, 0>{});
    if (qs + 1 < nqs) iter(qs + 1, std::integral_constant<int, 1>{});
  }
#undef BWD_GLDS

  // dK / dV of this q-head, rounded to bf16 like the per-head gradients of the reference's
  // repeat_kv + SDPA path; the finalize kernel sums the GQA group in fp32
  // (C layout: lane -> d, registers -> keys)
#pragma unroll
  for (int db = 0; db < NDB; ++db)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int k = kw + (r & 3) + 8 * (r >> 2) + 4 * hi;
      if (k < S) {
        const long off = ((long)b * S + k) * ldo + (long)h * D + db * 32 + l32;
        dk_part[off] = cvt1<E>(dk[db][r] * scale);
        dv_part[off] = cvt1<E>(dv[db][r]);
      }
    }
}

// One 4-column unit (row t, columns col .. col + 3) of the GQA fold / RoPE backward into dqkv
// (see flash_bwd_finalize_kernel): dQ from dq_acc (fp32) or rotated in place, dK / dV summed over
// the G q-head partials in head order (the same order wherever it runs: bit-reproducible).
template <class E>
__device__ __forceinline__ void fin_unit(const float* __restrict__ dq_acc, const bf16_t* __restrict__ dk_part,
                                         const bf16_t* __restrict__ dv_part, bf16_t* __restrict__ dqkv, long t,
                                         int col, int Hq, int Hkv, int D, const float* __restrict__ cos_t,
                                         const float* __restrict__ sin_t, int S, bool q_done = false) {
  const int G = Hq / Hkv;
  const int W = (Hq + 2 * Hkv) * D;
  float4 v;
  if (col < Hq * D) {
    if (dq_acc == nullptr) {  // dQ already written by the deterministic dQ kernel
      if (cos_t == nullptr || q_done) return;  // (q_done: rotated there too)
      const uint2 x = *reinterpret_cast<const uint2*>(dqkv + t * W + col);
      v = make_float4(u16f<E>(x.x), u16f<E>(x.x >> 16), u16f<E>(x.y), u16f<E>(x.y >> 16));
    } else {
      v = *reinterpret_cast<const float4*>(dq_acc + t * Hq * D + col);
    }
  } else {
    const bool isk = col < (Hq + Hkv) * D;
    const int c2 = col - (isk ? Hq * D : (Hq + Hkv) * D);
    const int kh = c2 / D, d = c2 % D;
    const bf16_t* src = (isk ? dk_part : dv_part) + t * Hq * D + (long)kh * G * D + d;
    v = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int r = 0; r < G; ++r) {
      const uint2 x = *reinterpret_cast<const uint2*>(src + r * D);
      v.x += u16f<E>(x.x); v.y += u16f<E>(x.x >> 16);
      v.z += u16f<E>(x.y); v.w += u16f<E>(x.y >> 16);
    }
  }
  if (cos_t != nullptr && col < (Hq + Hkv) * D) {
    // two interleaved pairs (col, col + 1), (col + 2, col + 3) of one head
    const int fi = (col % D) >> 1;
    const long pos = t % S;
    const float2 c = *reinterpret_cast<const float2*>(cos_t + pos * (D / 2) + fi);
    const float2 sn = *reinterpret_cast<const float2*>(sin_t + pos * (D / 2) + fi);
    const float a0 = v.x, b0 = v.y, a1 = v.z, b1 = v.w;
    // explicit fmas: the in-kernel fold (gqa_fold_rows) rounds identically
    v.x = fmaf(a0, c.x, b0 * sn.x);
    v.y = fmaf(-a0, sn.x, b0 * c.x);
    v.z = fmaf(a1, c.y, b1 * sn.y);
    v.w = fmaf(-a1, sn.y, b1 * c.y);
  }
  uint2 o;
  o.x = pk2<E>(v.x, v.y);
  o.y = pk2<E>(v.z, v.w);
  *reinterpret_cast<uint2*>(dqkv + t * W + col) = o;
}

// In-kernel GQA fold of the deterministic dK/dV kernel (no finalize pass): every (b, kv head, key
// tile) has G q-head blocks; each publishes its bf16 partial, fences, and bumps the tile's counter;
// the block that brings it to G folds the tile's rows (dK / dV over the G partials, RoPE backward
// of dK and of the group's dQ rows) and re-arms the counter for the next launch.
struct GqaFold {
  int* cnt;                // [B * Hkv * key tiles], zero between launches
  bf16_t* dqkv;            // [T, (Hq + 2 Hkv) D]
  const float* cos_t;      // RoPE tables or null
  const float* sin_t;
  int dbg;                 // timing experiments only: 1 no fold work, 2 no release fence
  int q_done;              // dQ already rotated by the dQ kernel
  int krot;                // no GQA (direct stores into dqkv): dK rotated back in the dK/dV kernel's row stores
};

// The fold of `rows` rows from t0 (one key tile of kv head kvh) by NT threads: 16-B units (8
// columns), U units in flight per thread (loads first, then the sums / rotations / stores: the
// per-unit load -> add -> store chains otherwise serialise on memory latency). Columns: the G
// q-heads' dQ (RoPE only, rotated in place), then dK, then dV of the kv head. Sums in head order.
template <class E, int D, int NT>
__device__ __forceinline__ void gqa_fold_rows(const bf16_t* __restrict__ dk_part, const bf16_t* __restrict__ dv_part,
                                              const GqaFold& f, long t0, int rows, int kvh, int G, int Hq, int Hkv,
                                              int S, int tid) {
  constexpr int U = 4, CU = D / 8;  // units per thread per pass, units per head row
  const long W = (long)(Hq + 2 * Hkv) * D;
  const int uq = f.cos_t != nullptr && !f.q_done ? G * CU : 0;
  const int upr = uq + 2 * CU;
  const int n = rows * upr;
  for (int base = 0; base < n; base += NT * U) {
    uint4 x[U][8];
    int rr[U], u[U];
#pragma unroll
    for (int j = 0; j < U; ++j) {
      const int i = base + j * NT + tid;
      rr[j] = i < n ? i / upr : -1;
      u[j] = i < n ? i - rr[j] * upr : 0;
      if (rr[j] < 0) continue;
      const long t = t0 + rr[j];
      if (u[j] < uq) {
        x[j][0] = *reinterpret_cast<const uint4*>(f.dqkv + t * W + (long)kvh * G * D + 8 * u[j]);
      } else {
        const bool isk = u[j] < uq + CU;
        const int c = 8 * (u[j] - uq - (isk ? 0 : CU));
        const bf16_t* src = (isk ? dk_part : dv_part) + t * Hq * D + (long)kvh * G * D + c;
#pragma unroll
        for (int r = 0; r < 8; ++r)
          if (r < G) x[j][r] = *reinterpret_cast<const uint4*>(src + r * D);
      }
    }
#pragma unroll
    for (int j = 0; j < U; ++j) {
      if (rr[j] < 0) continue;
      const long t = t0 + rr[j];
      float v[8];
      long col;
      bool rot;
      auto unpack_add = [&](const uint4& q, bool first) {
        const unsigned w4[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float lo = u16f<E>(w4[e]), hi = u16f<E>(w4[e] >> 16);
          v[2 * e] = first ? lo : v[2 * e] + lo;
          v[2 * e + 1] = first ? hi : v[2 * e + 1] + hi;
        }
      };
      if (u[j] < uq) {
        unpack_add(x[j][0], true);
        col = (long)kvh * G * D + 8 * u[j];
        rot = true;
      } else {
        const bool isk = u[j] < uq + CU;
        const int c = 8 * (u[j] - uq - (isk ? 0 : CU));
        // 0 + p0 + p1 + ... in head order, as flash_bwd_finalize_kernel
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = 0.f;
#pragma unroll
        for (int r = 0; r < 8; ++r)
          if (r < G) unpack_add(x[j][r], false);
        col = (isk ? (long)Hq * D : (long)(Hq + Hkv) * D) + (long)kvh * D + c;
        rot = isk && f.cos_t != nullptr;
      }
      if (rot) {
        const int fi = (int)(col % D) >> 1;
        const long pos = t % S;
        const float4 c4 = *reinterpret_cast<const float4*>(f.cos_t + pos * (D / 2) + fi);
        const float4 s4 = *reinterpret_cast<const float4*>(f.sin_t + pos * (D / 2) + fi);
        const float cc[4] = {c4.x, c4.y, c4.z, c4.w}, ss[4] = {s4.x, s4.y, s4.z, s4.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float a = v[2 * e], bb = v[2 * e + 1];
          v[2 * e] = fmaf(a, cc[e], bb * ss[e]);
          v[2 * e + 1] = fmaf(-a, ss[e], bb * cc[e]);
        }
      }
      uint4 o;
      o.x = pk2<E>(v[0], v[1]);
      o.y = pk2<E>(v[2], v[3]);
      o.z = pk2<E>(v[4], v[5]);
      o.w = pk2<E>(v[6], v[7]);
      *reinterpret_cast<uint4*>(f.dqkv + t * W + col) = o;
    }
  }
}

// ================================================================== backward dK/dV, slice pairs (deterministic)
// flash_bwd_kernel<D, 1> with TWO independent 32-query slices per loop iteration: S / dP
// of both slices are issued back to back, and in the steady state (both slices fully
// below the diagonal) the whole pair is one basic block, so the scheduler can run slice
// A's softmax VALU and dV / dK MFMAs while slice B's S / dP MFMAs are in flight (at one
// wave per SIMD there is no other wave to fill the MFMA pipe during a softmax phase).
// Q | dO pairs by LDS-DMA, double-buffered in two LDS objects (loop unrolled by two);
// the slices' lse / delta ride along in LDS (registers are the scarce resource here).
// SPLIT = 2: two half-blocks take alternate slice pairs of the same keys and add their dK / dV
// partials through LDS at the end (fixed order: bit-reproducible), halving the longest
// (first) key block's sweep.
// SD (self delta, the 3-kernel GQA backward): each slice's O rows come in by LDS-DMA beside its dO
// rows and every wave forms the slice's delta = rowsum(dO * O) itself (the dQ kernel's arithmetic,
// term for term: bitwise the same values), so this kernel runs FIRST and the dQ kernel after it
// folds the GQA partials (no finalize pass).
template <class E, int D, int NW = 4, int SPLIT = 1, bool SD = false>
__global__ __launch_bounds__(64 * NW * SPLIT, SPLIT == 1 ? 4 / NW : 8 / (NW * SPLIT)) void flash_bwd_dkdv2_kernel(
    const bf16_t* __restrict__ dO, const bf16_t* __restrict__ qk, const bf16_t* __restrict__ qkv,
    const float* __restrict__ lse2, const float* __restrict__ delta, bf16_t* __restrict__ dk_part,
    bf16_t* __restrict__ dv_part, long ldkv, int B, int S, int Hq, int Hkv, float sl2, float scale, long ldqk_,
    GqaFold fold, const bf16_t* __restrict__ O = nullptr) {
  constexpr int BK = 32 * NW, BQ = 32, KS = D / 16, NDB = D / 32;
  constexpr int QIMG = BQ * D * 2;          // one Q or dO slice
  constexpr int STO = (SD ? 3 : 2) * QIMG;  // lse[32] | delta[32] after Q | dO (| O)
  constexpr int SLOT = STO + 256;           // one slice
  __shared__ __attribute__((aligned(16))) char pb0[2 * SLOT * SPLIT];  // pair buffer 0: slice A | slice B
  __shared__ __attribute__((aligned(16))) char pb1[2 * SLOT * SPLIT];  // pair buffer 1 (per half-block)

  const int per = B * Hq;
  const int L = blockIdx.x;
  const int kt = L / per;  // key tile; kt = 0 has the most query slices -> launched first
  const int rem = L % per;
  const int b = rem / Hq;
  int h, kvh;
  map_head(rem % Hq, Hq, Hkv, h, kvh);

  const int tid = threadIdx.x, lane = tid & 63, l32 = lane & 31, hi = lane >> 5;
  const int hs = (tid >> 6) / NW, wave = (tid >> 6) % NW;  // half-block (pair parity), key group
  const int kb0 = kt * BK;
  const int kw = kb0 + wave * 32;  // this wave's first key
  const long ldqk = ldqk_, ldv = (long)(Hq + 2 * Hkv) * D, ldo = (long)Hq * D;
  const bf16_t* Qg = qk + (long)b * S * ldqk + (long)h * D;
  const bf16_t* Kg = qk + (long)b * S * ldqk + (long)(Hq + kvh) * D;
  const bf16_t* Vg = qkv + (long)b * S * ldv + (long)(Hq + Hkv + kvh) * D;
  const bf16_t* dOg = dO + (long)b * S * ldo + (long)h * D;
  const float* lseg = lse2 + ((long)b * Hq + h) * stat_stride(S);
  const float* delg = delta + ((long)b * Hq + h) * stat_stride(S);
  const bf16_t* Og = SD ? O + (long)b * S * ldo + (long)h * D : nullptr;

  typename FA<E>::v8 vf[KS], kf[KS];
  {
    const long key = min(kw + l32, S - 1);
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      vf[ks] = *reinterpret_cast<const typename FA<E>::v8*>(Vg + key * ldv + ks * 16 + hi * 8);
      kf[ks] = *reinterpret_cast<const typename FA<E>::v8*>(Kg + key * ldqk + ks * 16 + hi * 8);
    }
  }

  const int qs0 = kb0 / BQ;
  const int n = (S + BQ - 1) / BQ - qs0;  // slices of this key tile (>= 1)
  const int npairs = (n + 1) / 2;
  constexpr int GPW = QIMG / 1024 / NW;   // glds instructions per wave per image
  // pair p -> buffer: slices 2p (A) and 2p+1 (B, if any)
  auto dma = [&](int p, char* buf) __attribute__((always_inline)) {
#pragma unroll
    for (int half = 0; half < 2; ++half) {
      const int i = 2 * p + half;
      if (i < n) {  // block-uniform
        char* sl = buf + half * SLOT;
        const int q0 = (qs0 + i) * BQ;
        static_for<GPW>([&](auto I) {
          const int piece = wave * GPW + I;
          int r, c;
          lds_inv<D>(piece * 64 + lane, r, c);
          const long q = min(q0 + r, S - 1);
          glds16(Qg + q * ldqk + c * 8, sl + piece * 1024);
          glds16(dOg + q * ldo + c * 8, sl + QIMG + piece * 1024);
          if constexpr (SD) glds16(Og + q * ldo + c * 8, sl + 2 * QIMG + piece * 1024);
        });
        if (wave == half && lane < (SD ? 8 : 16)) {
          // lanes 0-7: lse rows q0..q0+31, lanes 8-15: delta (rows padded to 32: in bounds)
          const float* src = lane < 8 ? lseg + q0 + 4 * lane : delg + q0 + 4 * (lane - 8);
          glds16(src, sl + STO);
        }
      }
    }
  };

  f32x16_t dk[NDB], dv[NDB];
#pragma unroll
  for (int db = 0; db < NDB; ++db)
#pragma unroll
    for (int r = 0; r < 16; ++r) dk[db][r] = dv[db][r] = 0.f;

  const int key = kw + l32;
  auto sdp = [&](const char* sl, f32x16_t& sv, f32x16_t& dpv) __attribute__((always_inline)) {
    const char* qi = sl;
    const char* di = sl + QIMG;
#pragma unroll
    for (int r = 0; r < 16; ++r) sv[r] = dpv[r] = 0.f;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      sv = mfma32(ld_row<E, D>(qi, l32, 2 * ks + hi), kf[ks], sv);
      dpv = mfma32(ld_row<E, D>(di, l32, 2 * ks + hi), vf[ks], dpv);
    }
    if constexpr (SD) {
      // delta of query row l32 of the slice, as flash_bwd_dq_kernel forms it: this lane's half of
      // the dO . O dot product (columns 16 ks + 8 hi ..), plus lane ^ 32's; every wave writes the
      // same 32 values into the slot's delta row, read back by its own fin (LDS is in order per wave)
      const char* oi = sl + 2 * QIMG;
      float acc = 0.f;
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        const auto dv = ld_row<E, D>(di, l32, 2 * ks + hi);
        const auto ov = ld_row<E, D>(oi, l32, 2 * ks + hi);
        float x[8], y[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) x[j] = (float)dv[j];
#pragma unroll
        for (int j = 0; j < 8; ++j) y[j] = (float)ov[j];
#pragma unroll
        for (int j = 0; j < 8; ++j) acc += x[j] * y[j];
      }
      const float dl = acc + __shfl_xor(acc, 32, 64);
      if (hi == 0) reinterpret_cast<float*>(const_cast<char*>(sl) + STO)[BQ + l32] = dl;
    }
  };
  auto fin = [&](const char* sl, const int i, f32x16_t sv, f32x16_t dpv, auto MASKED)
      __attribute__((always_inline)) {
    constexpr bool MASK = decltype(MASKED)::value;
    const char* qi = sl;
    const char* di = sl + QIMG;
    const float* st = reinterpret_cast<const float*>(sl + STO);
    const int qb = (qs0 + i) * BQ;
    static_for<4>([&](auto G) {
      constexpr int g = G;
      const float4 l4 = *reinterpret_cast<const float4*>(st + 8 * g + 4 * hi);
      const float4 d4 = *reinterpret_cast<const float4*>(st + BQ + 8 * g + 4 * hi);
      const float lv[4] = {l4.x, l4.y, l4.z, l4.w};
      const float dv4[4] = {d4.x, d4.y, d4.z, d4.w};
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int r = 4 * g + t;
        float p = fast_exp2(fmaf(sv[r], sl2, -lv[t]));
        float ds = p * (dpv[r] - dv4[t]);
        if constexpr (MASK) {
          // also covers padded rows q >= S, whose lse / delta are uninitialised
          const int q = qb + 8 * g + 4 * hi + t;
          const bool off = key > q || q >= S;
          p = off ? 0.f : p;
          ds = off ? 0.f : ds;
        }
        dpv[r] = ds;
        sv[r] = p;
      }
    });
    const typename FA<E>::v8 pa[2] = {cvt8<E, 0>(sv), cvt8<E, 8>(sv)};
    const typename FA<E>::v8 da[2] = {cvt8<E, 0>(dpv), cvt8<E, 8>(dpv)};
#pragma unroll
    for (int ss = 0; ss < 2; ++ss)
#pragma unroll
      for (int db = 0; db < NDB; ++db) {
        dv[db] = mfma32(pa[ss], tr_frag<E, D>(di, 16 * ss, db * 32, lane), dv[db]);
        dk[db] = mfma32(da[ss], tr_frag<E, D>(qi, 16 * ss, db * 32, lane), dk[db]);
      }
  };
  // one slice, general case (inactive / masked / ragged)
  auto one = [&](const char* sl, const int i) __attribute__((always_inline)) {
    const int qb = (qs0 + i) * BQ;
    if (qb + BQ - 1 < kw) return;  // wave-uniform: all of the slice is above this wave's keys
    f32x16_t sv, dpv;
    sdp(sl, sv, dpv);
    if (kw + 31 > qb || qb + BQ > S)
      fin(sl, i, sv, dpv, std::true_type{});
    else
      fin(sl, i, sv, dpv, std::false_type{});
  };

  char* const b0 = pb0 + hs * 2 * SLOT;
  char* const b1 = pb1 + hs * 2 * SLOT;
  if (hs < npairs) dma(hs, b0);
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  // iteration it: this half-block's pair it * SPLIT + hs (both halves run the same number of
  // iterations so their barriers pair up; one may idle in the last)
  auto iter = [&](const int it, auto BUF) __attribute__((always_inline)) {
    constexpr int bb = decltype(BUF)::value;
    const int p = it * SPLIT + hs;
    char* cur = bb ? b1 : b0;
    if (p + SPLIT < npairs) dma(p + SPLIT, bb ? b0 : b1);
    const int ia = 2 * p, ib = 2 * p + 1;
    const int qa = (qs0 + ia) * BQ;
    // steady state: both slices entirely below this wave's diagonal and inside S
    if (p >= npairs) {
      // idle (this half-block has no pair left)
    } else if (ib < n && qa >= kw + 31 && qa + 2 * BQ <= S) {
      f32x16_t sa, dpa, sb, dpb;
      // the compiler's default schedule keeps the pair's phases apart; the IGLP
      // "DS + MFMA interleave" strategy spreads the LDS reads and the VALU between the
      // MFMAs (measured: 193.8 -> 182.4 us for the whole deterministic backward; iglp_opt(1)
      // 198.7 us)
      __builtin_amdgcn_iglp_opt(0);
      sdp(cur, sa, dpa);
      sdp(cur + SLOT, sb, dpb);
      fin(cur, ia, sa, dpa, std::false_type{});
      fin(cur + SLOT, ib, sb, dpb, std::false_type{});
    } else {
      one(cur, ia);
      if (ib < n) one(cur + SLOT, ib);
    }
    __builtin_amdgcn_s_waitcnt(0);  // this wave's DMA of pair p+1 has landed ...
    __syncthreads();                // ... and everyone's; nobody reads pair p any more
  };
  const int nit = (npairs + SPLIT - 1) / SPLIT;
  for (int it = 0; it < nit; it += 2) {
    iter(it, std::integral_constant<int, 0>{});
    if (it + 1 < nit) iter(it + 1, std::integral_constant<int, 1>{});
  }
  if constexpr (SPLIT == 2) {  // half-block 1 parks dK in pb0, dV in pb1; half-block 0 adds
    float* xk = reinterpret_cast<float*>(pb0) + (wave * 64 + lane);
    float* xv = reinterpret_cast<float*>(pb1) + (wave * 64 + lane);
    static_assert(NW * 64 * NDB * 16 * 4 <= 2 * SLOT * SPLIT, "merge buffer");
    if (hs == 1) {
#pragma unroll
      for (int db = 0; db < NDB; ++db)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          xk[(db * 16 + r) * NW * 64] = dk[db][r];
          xv[(db * 16 + r) * NW * 64] = dv[db][r];
        }
    }
    __syncthreads();
    if (hs == 1) return;
#pragma unroll
    for (int db = 0; db < NDB; ++db)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        dk[db][r] += xk[(db * 16 + r) * NW * 64];
        dv[db][r] += xv[(db * 16 + r) * NW * 64];
      }
  }

  // dK / dV of this q-head in bf16: per-q-head partials [T, Hq*D] (ldkv = Hq*D) that the
  // finalize kernel sums over the GQA group, or — without GQA (Hq == Hkv) — straight into the
  // K / V columns of dqkv (the pointers are offset by the host, ldkv = its row stride).
  // Staged through LDS (the pair buffers are free now): a lane holds one column of 16 key rows,
  // so storing from the accumulators takes 2-byte stores — 128 per lane, the kernel's tail; from
  // the staged rows every lane stores 16-byte row pieces (8 per array). Rows of D bf16, 16-byte
  // chunk c of row r at c ^ (r % CH).
  {
    constexpr int CH = D / 8;                 // 16-byte chunks per row
    constexpr int WB = 32 * D * 2 * 2;        // one wave's dK | dV rows
    constexpr int PB = 2 * SLOT * SPLIT;      // bytes of each pair buffer
    static_assert(2 * WB <= PB && NW <= 4, "dK/dV staging");
    __syncthreads();  // every wave is done with the pair buffers (and the SPLIT merge)
    char* const stg = (wave < 2 ? pb0 : pb1) + (wave & 1) * WB;
    auto at = [](int r, int d) { return r * (D * 2) + (((d >> 3) ^ (r % CH)) << 4) + (d & 7) * 2; };
#pragma unroll
    for (int db = 0; db < NDB; ++db)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int kr = (r & 3) + 8 * (r >> 2) + 4 * hi;
        const int d = db * 32 + l32;
        *reinterpret_cast<bf16_t*>(stg + at(kr, d)) = cvt1<E>(dk[db][r] * scale);
        *reinterpret_cast<bf16_t*>(stg + 32 * D * 2 + at(kr, d)) = cvt1<E>(dv[db][r]);
      }
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's staging writes landed
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int it = 0; it < 32 * CH / 64; ++it) {
      const int i = it * 64 + lane, r = i / CH, c = i % CH;
      const int k = kw + r;
      if (k < S) {
        const int so = r * (D * 2) + ((c ^ (r % CH)) << 4);
        const long off = ((long)b * S + k) * ldkv + (long)h * D + c * 8;
        uint4 kv = *reinterpret_cast<const uint4*>(stg + so);
        if (fold.krot) {  // (uniform) RoPE backward of the 4 pairs of this dK chunk, as rope_bwd_ does it
          const float4 c4 = *reinterpret_cast<const float4*>(fold.cos_t + (long)k * (D / 2) + c * 4);
          const float4 s4 = *reinterpret_cast<const float4*>(fold.sin_t + (long)k * (D / 2) + c * 4);
          const float cc[4] = {c4.x, c4.y, c4.z, c4.w}, ss[4] = {-s4.x, -s4.y, -s4.z, -s4.w};
          float x[8], y[8];
          unpack8e<E>(kv, x);
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const float a = x[2 * q], bb = x[2 * q + 1];
            y[2 * q] = a * cc[q] - bb * ss[q];
            y[2 * q + 1] = a * ss[q] + bb * cc[q];
          }
          kv = pack8e<E>(y);
        }
        *reinterpret_cast<uint4*>(dk_part + off) = kv;
        *reinterpret_cast<uint4*>(dv_part + off) = *reinterpret_cast<const uint4*>(stg + 32 * D * 2 + so);
      }
    }
  }

  if (fold.cnt != nullptr) {
    // (SPLIT = 2: half-block 1 has exited; the barriers count the 64 * NW threads left)
    __shared__ int s_last;
    const int G = Hq / Hkv;
    const int ci = (b * Hkv + kvh) * (int)(gridDim.x / per) + kt;
    // release only (L2 write-back, no invalidate): an acquire here would drop every block's L2
    // working set; only the folding block needs one
    if (fold.dbg != 2) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");  // partial visible device-wide
    __syncthreads();
    if (tid == 0) s_last = atomicAdd(fold.cnt + ci, 1) == G - 1;
    __syncthreads();
    if (!s_last) return;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");  // the other G - 1 partials
    if (tid == 0) fold.cnt[ci] = 0;
    if (fold.dbg != 1)
      gqa_fold_rows<E, D, 64 * NW>(dk_part, dv_part, fold, (long)b * S + kb0, min(BK, S - kb0), kvh, G, Hq, Hkv, S,
                                 tid);
  }
}

// ================================================================== backward dQ (deterministic)
// Q-major like the forward: per wave 32 query rows, sweep 64-key tiles up to the
// diagonal; S^T = K Q^T and dP^T = V dO^T (A = K / V rows from LDS, B = Q^T / dO^T
// in VGPRs), dS^T = P^T (dP^T - delta) with P = exp2(S^T*c - lse2) (the query is on
// the lane, so lse/delta are per-lane scalars), dQ^T += K^T dS^T (A = K^T through
// transposed LDS reads, B = dS^T straight from the accumulators). Every dQ element
// is produced by exactly one wave in a fixed order: no atomics, bit-reproducible.
// Used with flash_bwd_kernel<D, 1> (dK/dV only) for --deterministic runs.
// SPLIT = 2 (small grids, see flash_bwd): as the forward's key split, two half-blocks sweep
// the even / odd key tiles of the same queries and add their dQ partials through LDS (in a
// fixed order: still bit-reproducible).
// O != null: the kernel forms delta = rowsum(dO * O) itself (each lane pair already holds its
// query's dO row) and publishes it for the dK/dV kernel that runs after it — the separate
// flash_bwd_pre pass and its second read of dO are gone.
template <class E, int D, int NW = 4, int SPLIT = 1>
__global__ __launch_bounds__(64 * NW * SPLIT, SPLIT == 1 ? 4 / NW : 8 / (NW * SPLIT)) void flash_bwd_dq_kernel(
    const bf16_t* __restrict__ dO, const bf16_t* __restrict__ qk, const bf16_t* __restrict__ qkv,
    const float* __restrict__ lse2, float* __restrict__ delta, bf16_t* __restrict__ dqkv, int B,
    int S, int Hq, int Hkv, float sl2, float scale, long ldqk_, const bf16_t* __restrict__ O,
    const float* __restrict__ cos_t, const float* __restrict__ sin_t,
    const bf16_t* __restrict__ dk_part = nullptr, const bf16_t* __restrict__ dv_part = nullptr) {
  constexpr int BM = 32 * NW, BN = 64, KS = D / 16, NDB = D / 32;
  constexpr int TILE = BN * D * 2;
  // K | V tiles arrive by LDS-DMA (no staging VGPRs held across the compute: at one wave
  // per SIMD the register-staged prefetch pushed the dQ accumulators through AGPR copies
  // every tile). Two separate LDS objects + a loop unrolled by two: every row read names a
  // buffer the in-flight DMA provably does not write, so the compiler does not drain the
  // prefetch before them (it still does before the first transposed ds_read_b64_tr_b16 of a
  // tile; asm reads that avoid it measured no gain: profiles/r2_flash_d64_forward_ab.log).
  __shared__ __attribute__((aligned(16))) char kv0[2 * TILE * SPLIT];
  __shared__ __attribute__((aligned(16))) char kv1[2 * TILE * SPLIT];

  const int nqt = (S + BM - 1) / BM;
  const int per = B * Hq;
  const int L = blockIdx.x;
  const int qt = nqt - 1 - L / per;
  const int rem = L % per;
  const int b = rem / Hq;
  int h, kvh;
  map_head(rem % Hq, Hq, Hkv, h, kvh);

  const int tid = threadIdx.x, lane = tid & 63, l32 = lane & 31, hi = lane >> 5;
  const int half = (tid >> 6) / NW, wave = (tid >> 6) % NW;  // key-tile parity, query group
  const int q0 = qt * BM + wave * 32;
  const int qrow = q0 + l32;
  const long ldqk = ldqk_, ldv = (long)(Hq + 2 * Hkv) * D, ldo = (long)Hq * D;
  const bf16_t* Qg = qk + (long)b * S * ldqk + (long)h * D;
  const bf16_t* Kg = qk + (long)b * S * ldqk + (long)(Hq + kvh) * D;
  const bf16_t* Vg = qkv + (long)b * S * ldv + (long)(Hq + Hkv + kvh) * D;
  const bf16_t* dOg = dO + (long)b * S * ldo + (long)h * D;

  typename FA<E>::v8 qf[KS], df[KS];
  const long qr = min(qrow, S - 1);
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    qf[ks] = *reinterpret_cast<const typename FA<E>::v8*>(Qg + qr * ldqk + ks * 16 + hi * 8);
    df[ks] = *reinterpret_cast<const typename FA<E>::v8*>(dOg + qr * ldo + ks * 16 + hi * 8);
  }
  const float lq = lse2[((long)b * Hq + h) * stat_stride(S) + qr];
  float dlq;
  if (O != nullptr) {  // uniform
    // delta of this lane's query: its half of the dO . O dot product, plus the other half
    // from lane ^ 32 (same query, the other 8 of every 16 columns); fp32 like flash_bwd_pre
    const bf16_t* Og = O + (long)b * S * ldo + (long)h * D + qr * ldo;
    float acc = 0.f;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      float x[8], y[8];
      ld8<E>(Og + ks * 16 + hi * 8, y);
      const auto dv = df[ks];
#pragma unroll
      for (int j = 0; j < 8; ++j) x[j] = (float)dv[j];
#pragma unroll
      for (int j = 0; j < 8; ++j) acc += x[j] * y[j];
    }
    dlq = acc + __shfl_xor(acc, 32, 64);
    if (half == 0 && hi == 0 && qrow < S) delta[((long)b * Hq + h) * stat_stride(S) + qrow] = dlq;
  } else {
    dlq = delta[((long)b * Hq + h) * stat_stride(S) + qr];
  }

  const int kend = min((qt + 1) * BM, S);
  const int ntiles = (kend + BN - 1) / BN;
  constexpr int GPW = TILE / 1024 / NW;  // glds instructions per wave per image
  // tile KT -> buffer BUF: each lane moves one 16-B chunk; the swizzle is on the source
  auto dma = [&](int KT, auto BUF) {
    char* kb_ = (decltype(BUF)::value ? kv1 : kv0) + half * 2 * TILE;
    static_for<GPW>([&](auto I) {
      const int piece = wave * GPW + I;
      int r, c;
      lds_inv<D>(piece * 64 + lane, r, c);
      const long key = min(KT * BN + r, S - 1);
      glds16(Kg + key * ldqk + c * 8, kb_ + piece * 1024);
      glds16(Vg + key * ldv + c * 8, kb_ + TILE + piece * 1024);
    });
  };

  if (half < ntiles) dma(half, std::integral_constant<int, 0>{});
  // Materialise the Q / dO fragments and row statistics before the loop: left pending,
  // the compiler's waits for them inside the loop would drain the next tile's prefetch.
  asm volatile("" ::"v"(lq), "v"(dlq));
  static_for<KS>([&qf, &df](auto I) {
    asm volatile("" ::"v"(__builtin_bit_cast(u32x4, qf[I])), "v"(__builtin_bit_cast(u32x4, df[I])));
  });
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();

  f32x16_t dq[NDB];
#pragma unroll
  for (int db = 0; db < NDB; ++db)
#pragma unroll
    for (int r = 0; r < 16; ++r) dq[db][r] = 0.f;

  auto iter = [&](const int it, auto CUR) {  // this half's key tile it * SPLIT + half
    constexpr int cur = decltype(CUR)::value;
    const int kt = it * SPLIT + half;
    if (kt + SPLIT < ntiles) dma(kt + SPLIT, std::integral_constant<int, cur ^ 1>{});
    const char* kb = (cur ? kv1 : kv0) + half * 2 * TILE;
    const char* vb = kb + TILE;
    const int k0 = kt * BN;
    const bool v0 = k0 <= q0 + 31;
    const bool v1 = k0 + 32 <= q0 + 31;
    auto tile = [&](auto MASKED) {
      constexpr bool MASK = decltype(MASKED)::value;
      f32x16_t sc[2], dp[2];
#pragma unroll
      for (int j = 0; j < 2; ++j) {
#pragma unroll
        for (int r = 0; r < 16; ++r) sc[j][r] = dp[j][r] = 0.f;
        if (!MASK || j == 0 || v1) {
#pragma unroll
          for (int ks = 0; ks < KS; ++ks) {
            sc[j] = mfma32(ld_row<E, D>(kb, j * 32 + l32, 2 * ks + hi), qf[ks], sc[j]);
            dp[j] = mfma32(ld_row<E, D>(vb, j * 32 + l32, 2 * ks + hi), df[ks], dp[j]);
          }
        }
      }
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          float p = fast_exp2(fmaf(sc[j][r], sl2, -lq));
          if constexpr (MASK) {
            const int key = k0 + j * 32 + (r & 3) + 8 * (r >> 2) + 4 * hi;
            if ((j == 1 && !v1) || key > qrow || qrow >= S) p = 0.f;
          }
          sc[j][r] = p * (dp[j][r] - dlq);
        }
      const typename FA<E>::v8 d00 = cvt8<E, 0>(sc[0]), d01 = cvt8<E, 8>(sc[0]);
      const typename FA<E>::v8 d10 = cvt8<E, 0>(sc[1]), d11 = cvt8<E, 8>(sc[1]);
#pragma unroll
      for (int db = 0; db < NDB; ++db) {
        dq[db] = mfma32(tr_frag<E, D>(kb, 0, db * 32, lane), d00, dq[db]);
        dq[db] = mfma32(tr_frag<E, D>(kb, 16, db * 32, lane), d01, dq[db]);
      }
      if (!MASK || v1) {
#pragma unroll
        for (int db = 0; db < NDB; ++db) {
          dq[db] = mfma32(tr_frag<E, D>(kb, 32, db * 32, lane), d10, dq[db]);
          dq[db] = mfma32(tr_frag<E, D>(kb, 48, db * 32, lane), d11, dq[db]);
        }
      }
    };
    if (v0 && kt < ntiles) {
      // rows >= S (ragged last tile) take the masked path too
      if (k0 + BN - 1 > q0 || q0 + 31 >= S)
        tile(std::true_type{});
      else
        tile(std::false_type{});
    }
    __builtin_amdgcn_s_waitcnt(0);  // this wave's DMA of tile kt+1 has landed ...
    __syncthreads();                // ... and everyone's; nobody reads tile kt any more
  };
  const int nit = (ntiles + SPLIT - 1) / SPLIT;
  for (int it = 0; it < nit; it += 2) {
    iter(it, std::integral_constant<int, 0>{});
    if (it + 1 < nit) iter(it + 1, std::integral_constant<int, 1>{});
  }
  if constexpr (SPLIT == 2) {  // odd-tile half parks its dQ in LDS, the even half adds it
    float* xq = reinterpret_cast<float*>(kv0) + (wave * 64 + lane);
    static_assert(NW * 64 * NDB * 16 * 4 <= 2 * TILE * SPLIT, "merge buffer");
    if (half == 1) {
#pragma unroll
      for (int db = 0; db < NDB; ++db)
#pragma unroll
        for (int r = 0; r < 16; ++r) xq[(db * 16 + r) * NW * 64] = dq[db][r];
    }
    __syncthreads();
    if (half == 1) return;
#pragma unroll
    for (int db = 0; db < NDB; ++db)
#pragma unroll
      for (int r = 0; r < 16; ++r) dq[db][r] += xq[(db * 16 + r) * NW * 64];
  }

  if (cos_t == nullptr) {
    store_row16<E, NDB>(dqkv + ((long)b * S + min(qrow, S - 1)) * ldv + (long)h * D, hi, qrow < S,
                        [&](int db, int i) { return dq[db][i] * scale; });
  } else {
    // RoPE backward of dQ here (reference model.py:100-126 transposed: the interleaved pair
    // (x0, x1) times cis(-theta)): a lane's 4 consecutive columns are two whole pairs, so the
    // rotation is in-lane, in fp32 before the one rounding; the finalize pass skips the Q columns
    const long pos = min(qrow, S - 1);
    store_row16<E, NDB>(dqkv + ((long)b * S + pos) * ldv + (long)h * D, hi, qrow < S, [&](int db, int i) {
      const int i0 = i & ~1;
      const float a0 = dq[db][i0] * scale, b0 = dq[db][i0 + 1] * scale;
      // the lane's 4 columns are 2 whole pairs: one float2 of cos / sin each (the 4 calls of a
      // group load the same addresses, merged by the compiler) instead of 2 scalar loads per element
      const int fb = (db * 32 + 8 * (i >> 2) + 4 * hi) >> 1;
      const float2 c2 = *reinterpret_cast<const float2*>(cos_t + pos * (D / 2) + fb);
      const float2 s2 = *reinterpret_cast<const float2*>(sin_t + pos * (D / 2) + fb);
      const float c = (i & 2) ? c2.y : c2.x, sn = (i & 2) ? s2.y : s2.x;
      return (i & 1) ? fmaf(-a0, sn, b0 * c) : fmaf(a0, c, b0 * sn);
    });
  }

  if (dk_part != nullptr) {  // (uniform) the 3-kernel GQA backward: the dK/dV kernel ran first
    // Fold of its per-q-head partials: this block takes key rows [qt BM, +BM) of kv head kvh and
    // column slice gi (D / G columns) of dK and dV: the sum over the G q-heads in head order, dK
    // rotated back (RoPE), as flash_bwd_finalize_kernel / gqa_fold_rows compute it (bitwise).
    // (SPLIT = 2: half-block 1 has returned; the 64 NW threads of half 0 do it.)
    const int G = Hq / Hkv, gi = h - kvh * G;
    const int cps = D / G / 8;  // 16-B chunks per column slice
    const int r0 = qt * BM, nr = min(BM, S - r0);
    const long W = (long)(Hq + 2 * Hkv) * D;
    const int n = nr * 2 * cps;
    for (int i = tid; i < n; i += 64 * NW) {
      const int row = i / (2 * cps), u = i - row * 2 * cps;
      const bool isk = u < cps;
      const int c = (gi * cps + (isk ? u : u - cps)) * 8;  // first column within the head
      const long t = (long)b * S + r0 + row;
      const bf16_t* src = (isk ? dk_part : dv_part) + t * Hq * D + (long)kvh * G * D + c;
      float v[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = 0.f;
      for (int g = 0; g < G; ++g) {
        const uint4 q = *reinterpret_cast<const uint4*>(src + g * D);
        const unsigned w4[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          v[2 * e] = v[2 * e] + u16f<E>(w4[e]);
          v[2 * e + 1] = v[2 * e + 1] + u16f<E>(w4[e] >> 16);
        }
      }
      if (isk && cos_t != nullptr) {
        const long pos = r0 + row;
        const float4 c4 = *reinterpret_cast<const float4*>(cos_t + pos * (D / 2) + (c >> 1));
        const float4 s4 = *reinterpret_cast<const float4*>(sin_t + pos * (D / 2) + (c >> 1));
        const float cc[4] = {c4.x, c4.y, c4.z, c4.w}, ss[4] = {s4.x, s4.y, s4.z, s4.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float a = v[2 * e], bb = v[2 * e + 1];
          v[2 * e] = fmaf(a, cc[e], bb * ss[e]);
          v[2 * e + 1] = fmaf(-a, ss[e], bb * cc[e]);
        }
      }
      uint4 o;
      o.x = pk2<E>(v[0], v[1]);
      o.y = pk2<E>(v[2], v[3]);
      o.z = pk2<E>(v[4], v[5]);
      o.w = pk2<E>(v[6], v[7]);
      *reinterpret_cast<uint4*>(dqkv + t * W + (isk ? (long)Hq * D : (long)(Hq + Hkv) * D) + (long)kvh * D + c) = o;
    }
  }
}

// dqkv[:, q | k | v] = bf16(dQ), bf16(sum_G dK_part), bf16(sum_G dV_part).
// cos_t != null: the Q and K columns are also rotated back (RoPE backward, reference
// model.py:100-126 transposed: the interleaved pair (x0, x1) times cis(-theta)), so dqkv is the
// gradient of the unrotated projection and no separate rope_bwd pass runs; dQ written by the
// deterministic dQ kernel is rotated in place. The deterministic path folds inside the dK/dV kernel
// (fin_unit from its last GQA block); this pass remains for the other backward variants.
template <class E>
__global__ __launch_bounds__(256) void flash_bwd_finalize_kernel(
    const float* __restrict__ dq_acc, const bf16_t* __restrict__ dk_part,
    const bf16_t* __restrict__ dv_part, bf16_t* __restrict__ dqkv, long T, int Hq, int Hkv, int D,
    const float* __restrict__ cos_t, const float* __restrict__ sin_t, int S, int q_done) {
  const int W = (Hq + 2 * Hkv) * D;
  // q_done: the dQ columns are final (rotated by the dQ kernel): only the K / V columns remain
  const int c0 = q_done ? Hq * D / 4 : 0;
  const int vpr = W / 4 - c0;
  const long total = T * vpr;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const long t = i / vpr;
    fin_unit<E>(dq_acc, dk_part, dv_part, dqkv, t, (int)(i - t * vpr + c0) * 4, Hq, Hkv, D, cos_t, sin_t, S,
                q_done != 0);
  }
}

// Forward key split (see flash_fwd_kernel): -1 auto, 0 off, 1 on (flash_set_fwd_split, for A/B;
// tests/test_flash_attn_gpu.py).
int g_fwd_split = -1;

// Software-pipelined forward (flash_fwd_pipe_kernel) for the unsplit grids: >= 1 on, 0 off
// (flash_set_fwd_pipe, for A/B). (A balanced variant — one 8-wave block per query-tile pair, the
// long tile's keys split between the halves and merged in LDS — ran slower: 60.0 vs 53.3 us at
// S = 2048, profiles/r3_flash_fwd_pipe.log.)
int g_fwd_pipe = 1;

// Per-block timestamps of the pipelined forward (int64 [grid, 8]; flash_set_fwd_prof, for
// scripts/flash_fwd_timeline.py); nullptr = off. (Measured with it, round 5: running the heavy
// query tiles as two key halves merged through an agent-scope hand-off made the S = 2048 layer
// slower, 49.2 -> 63.6 us: the extra blocks' prologue (~4-5 us of load latency each) and the
// hand-off (epilogue 2.0 -> 6.3 us) cost more than the balance gained; at S = 8192 it balanced
// the CUs but the span stayed 746 us. profiles/r5_flash_fwd_timeline_khalf.log.)
long long* g_fwd_prof = nullptr;
long g_fwd_prof_rows = 0;  // rows of the probe buffer (checked against the grid at launch)

// dQ key split (see flash_bwd_dq_kernel): -1 default (on), 0 off, 1 on (flash_set_dq_split, for A/B).
int g_dq_split = -1;

// dK/dV split of the slice-pair kernel: -1 auto, 0 off, 1 on (flash_set_kv_split, for A/B).
int g_kv_split = -1;

// Deterministic backward, dK/dV stage: the slice-pair kernel (default) or the one-slice
// flash_bwd_kernel<D, 1> (flash_set_dkdv2, for A/B); the slice-pair kernel also for head_dim 64:
// g_dkdv2_64 (measured slower there, off).
bool g_dkdv2 = true;
bool g_dkdv2_64 = false;

// GQA fold of the deterministic backward in the separate finalize pass (default) or inside the
// dK/dV kernel by each key tile's last q-head block (flash_set_bwd_fold).
// The in-kernel fold saves the launch but measured slower at the 8B layer (S = 2048, 32/8 heads,
// RoPE): 296-307 us vs 175-193 us for the whole backward; its device-scope release fences and
// counters alone cost ~16 us over the finalize variant without any fold work, and the folds run
// as a 128-block tail behind the heaviest key tiles (profiles/r4_flash_gqa_fold_probe.log).
bool g_bwd_fold = false;

// No-GQA backward (GPT-2-sized presets): dQ rotated in the dQ kernel's store and dK in the dK/dV
// kernel's, so no separate rope_bwd_ pass (3 kernels per layer); flash_set_direct_rope(false): the
// pass after the two kernels (A/B).
// GQA deterministic backward in 3 kernels (FT_FLASH_FOLD3=1 / flash_set_fold3(true)): the dK/dV
// kernel first, forming delta itself from O (SD), then the dQ kernel, which also folds the GQA
// partials (no finalize pass). Bitwise equal to the default 4-kernel order (dQ, dK/dV, finalize) but
// slower at the 8B layer: 200.8 vs 165.7 us -- every wave of the dK/dV kernel forms its slices'
// deltas on the critical path (88.6 -> 120.7 us), and the fold in the dQ kernel costs what the
// finalize pass did (+11.6 vs 9.6 us) (profiles/r6/flash_fold3_ab.log). Off by default.
bool g_fold3 = [] {
  const char* e = std::getenv("FT_FLASH_FOLD3");
  return e != nullptr && std::atoi(e) != 0;
}();

bool g_direct_rope = [] {
  const char* e = std::getenv("FT_FLASH_DIRECT_ROPE");
  return e == nullptr || std::atoi(e) != 0;
}();

// The fold's per-tile arrival counters: one zeroed int32 buffer per device, grown on demand and
// kept (each tile's last block re-arms its counter, so the buffer is zero between launches). One
// backward in flight per device at a time (the training step's single compute stream). Under
// stream capture a buffer that would have to be (re)allocated is not: the caller falls back to
// the finalize pass.
int* fold_counters(const c10::Device& dev, long n) {
  static std::mutex mu;
  static std::map<int, at::Tensor> bufs;
  std::lock_guard<std::mutex> lock(mu);
  at::Tensor& b = bufs[dev.index()];
  if (!b.defined() || b.numel() < n) {
    hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(ft_stream(), &st) != hipSuccess || st != hipStreamCaptureStatusNone) return nullptr;
    b = at::zeros({std::max(n, 4096L)}, at::TensorOptions().device(dev).dtype(at::kInt));
  }
  return b.data_ptr<int>();
}

// Waves (32 query or key rows each) per attention block: 2 when 4-wave blocks would leave
// most of the 256 CUs idle (fewer than 512 blocks; head_dim 64 — the GPT-2-sized presets:
// 12 / 16 heads x 16 tiles = 192 / 256 blocks at S = 2048), else 4.
// The forward keeps 4-wave blocks (2 waves: 32.0 -> 36.6 us on GPT-2-small's layer); the
// backward's dK/dV + dQ kernels gain (112.8 -> 94.2 us; 118.2 -> 99.2 us at 16 heads),
// profiles/r2_flash_small_heads.log.
static const bool g_force_nw4 = false;
int waves_per_block(long S, long B, long Hq, long D) {
  if (g_force_nw4) return 4;
  return (D == 64 && ((S + 127) / 128) * B * Hq < 512) ? 2 : 4;
}

void check_inputs(const at::Tensor& qk, const at::Tensor& qkv, int64_t S, int64_t Hq, int64_t Hkv,
                  int64_t D) {
  FT_CHECK_CUDA(qk);
  TORCH_CHECK(qk.scalar_type() == at::kBFloat16 || qk.scalar_type() == at::kHalf,
              "flash: qk must be bf16 or fp16 (fp32 models use flash_f32_*)");
  TORCH_CHECK(qkv.scalar_type() == qk.scalar_type(), "flash: qk / qkv dtype mismatch");
  FT_CHECK_CONTIG(qk);
  FT_CHECK_CONTIG(qkv);
  TORCH_CHECK(D == 64 || D == 128, "flash: head_dim must be 64 or 128");
  TORCH_CHECK(Hq % Hkv == 0, "flash: Hq must be a multiple of Hkv");
  // qk: the rotated [T, (Hq + Hkv) D] Q/K buffer, or the qkv buffer itself when the QKV projection
  // rotated Q/K in its epilogue (gemm_qkv_rope_w4); the kernels take its row stride
  TORCH_CHECK(qk.size(-1) == (Hq + Hkv) * D || qk.size(-1) == (Hq + 2 * Hkv) * D, "flash: qk width");
  TORCH_CHECK(qkv.size(-1) == (Hq + 2 * Hkv) * D, "flash: qkv width");
  TORCH_CHECK(qk.size(0) == qkv.size(0) && qk.size(0) % S == 0, "flash: rows");
}

}  // namespace

// Returns (o [T, Hq*D] bf16, lse2 [B, Hq, Sp] fp32 with Sp = S rounded up to 32 (entries
// >= S unused); lse2 = log2 of the softmax denominator in the exp2 domain, i.e.
// P = exp2(s * scale * log2e - lse2)).
std::tuple<at::Tensor, at::Tensor> flash_fwd(const at::Tensor& qk, const at::Tensor& qkv,
                                             int64_t S, int64_t Hq, int64_t Hkv, int64_t D) {
  check_inputs(qk, qkv, S, Hq, Hkv, D);
  const int T = qk.size(0);
  const int B = T / S;
  const at::DeviceGuard guard(qk.device());
  auto out = at::empty({T, Hq * D}, qk.options());
  auto lse = at::empty({B, Hq, (long)stat_stride(S)}, qk.options().dtype(at::kFloat));
  const float sl2 = LOG2E_F / std::sqrt((float)D);
  const long ldqk = qk.size(-1);
  const int nw = 4;  // see waves_per_block
  const int nqt = (S + 32 * nw - 1) / (32 * nw);
  // key-split blocks when the grid is at most one block per CU (FT_FLASH_FWD_SPLIT=0/1 forces)
  const bool split = g_fwd_split >= 0 ? g_fwd_split == 1 : (long)nqt * B * Hq <= 256;
  dim3 grid(nqt * B * Hq), block(64 * nw * (split ? 2 : 1));
#define FT_FWD(DD, SP)                                                                             \
  hipLaunchKernelGGL((flash_fwd_kernel<E, DD, 4, SP>), grid, block, 0, ft_stream(), cptr<bf16_t>(qk), \
                     cptr<bf16_t>(qkv), mptr<bf16_t>(out), mptr<float>(lse), B, (int)S, (int)Hq,   \
                     (int)Hkv, sl2, ldqk)
#define FT_FWD_PIPE(DD)                                                                            \
  hipLaunchKernelGGL((flash_fwd_pipe_kernel<E, DD, 4>), grid, block, 0, ft_stream(), cptr<bf16_t>(qk), \
                     cptr<bf16_t>(qkv), mptr<bf16_t>(out), mptr<float>(lse), B, (int)S, (int)Hq,   \
                     (int)Hkv, sl2, ldqk, g_fwd_prof)
  const bool pipe = !split && g_fwd_pipe >= 1;
  TORCH_CHECK(g_fwd_prof == nullptr || !pipe || (long)grid.x <= g_fwd_prof_rows,
              "flash_set_fwd_prof: the buffer needs ", grid.x, " rows of 8 int64");
  FT_DISPATCH_E16(qk.scalar_type(), {
    if (D == 128) {
      if (split) FT_FWD(128, 2); else if (pipe) FT_FWD_PIPE(128); else FT_FWD(128, 1);
    } else {
      if (split) FT_FWD(64, 2); else if (pipe) FT_FWD_PIPE(64); else FT_FWD(64, 1);
    }
  });
#undef FT_FWD
#undef FT_FWD_PIPE
  FT_LAUNCH_CHECK();
  return {out, lse};
}

// Returns dqkv [T, (Hq+2Hkv)*D] bf16 (dQ/dK in the rotated frame; RoPE backward follows).
// rope.hip: in-place RoPE backward on the Q / K columns of dqkv
void rope_bwd_(const at::Tensor& dqkv, const at::Tensor& cos_t, const at::Tensor& sin_t, int64_t seq_len,
               int64_t hq, int64_t hkv, int64_t d);

// cos / sin given: the returned dQ / dK are rotated back (the gradient of the UNROTATED
// projection), inside the pass that folds the GQA dK / dV partials.
at::Tensor flash_bwd(const at::Tensor& dout, const at::Tensor& qk, const at::Tensor& qkv,
                     const at::Tensor& out, const at::Tensor& lse, int64_t S, int64_t Hq,
                     int64_t Hkv, int64_t D, int64_t mode, const std::optional<at::Tensor>& cos_t,
                     const std::optional<at::Tensor>& sin_t) {
  check_inputs(qk, qkv, S, Hq, Hkv, D);
  FT_CHECK_CONTIG(dout);
  FT_CHECK_CONTIG(out);
  const int T = qk.size(0);
  const int B = T / S;
  TORCH_CHECK(dout.numel() == (long)T * Hq * D && out.numel() == (long)T * Hq * D, "flash_bwd: o shape");
  TORCH_CHECK(lse.numel() == (long)B * Hq * stat_stride(S), "flash_bwd: lse shape");
  const at::DeviceGuard guard(qk.device());
  auto f32 = qk.options().dtype(at::kFloat);
  auto delta = at::empty({B, Hq, (long)stat_stride(S)}, f32);
  // mode 0: dQ by fp32 atomics in the KV-major kernel (fastest);
  // mode 1: deterministic — KV kernel without dQ + Q-major dQ kernel (no atomics);
  // mode 2: timing experiment only (racy dQ stores).
  const bool det = mode == 1;
  at::Tensor dq_acc = det ? at::Tensor() : (mode == 2 ? at::empty({T, Hq * D}, f32) : at::zeros({T, Hq * D}, f32));
  const int nw_ = waves_per_block(S, B, Hq, D);
  // slice-pair dK/dV kernel in the deterministic mode (else the one-slice flash_bwd_kernel)
  const bool use_dkdv2 = det && (D == 128 ? (g_dkdv2 && nw_ == 4) : (nw_ == 2 || g_dkdv2_64));
  // no GQA: that kernel writes dK / dV into dqkv itself, dQ comes from the dQ kernel, so the
  // finalize pass (and the partial buffers) are skipped
  const bool direct = use_dkdv2 && Hq == Hkv;
  auto dqkv = at::empty({T, (Hq + 2 * Hkv) * D}, qk.options());
  at::Tensor dk_part = direct ? at::Tensor() : at::empty({T, Hq * D}, qk.options());
  at::Tensor dv_part = direct ? at::Tensor() : at::empty({T, Hq * D}, qk.options());
  bf16_t* dkp = direct ? mptr<bf16_t>(dqkv) + (long)Hq * D : mptr<bf16_t>(dk_part);
  bf16_t* dvp = direct ? mptr<bf16_t>(dqkv) + (long)(Hq + Hkv) * D : mptr<bf16_t>(dv_part);
  const long ldkv = direct ? (long)(Hq + 2 * Hkv) * D : (long)Hq * D;
  const bool rope = cos_t.has_value() && cos_t->defined();
  if (rope) {
    TORCH_CHECK(sin_t.has_value() && sin_t->defined(), "flash_bwd: cos without sin");
    FT_CHECK_F32((*cos_t));
    FT_CHECK_F32((*sin_t));
    FT_CHECK_CONTIG((*cos_t));
    FT_CHECK_CONTIG((*sin_t));
    TORCH_CHECK(cos_t->size(0) >= S && cos_t->size(1) == D / 2 && sin_t->sizes() == cos_t->sizes(),
                "flash_bwd: rope tables must be [>= S, D / 2]");
  }
  const float sl2 = LOG2E_F / std::sqrt((float)D);
  const float scale = 1.f / std::sqrt((float)D);
  const long ldqk = qk.size(-1);
  const long rows = (long)T * Hq;
  // GQA fold inside the deterministic dK/dV kernel (no finalize launch): its tile counters
  static const int fold_dbg = [] {
    return 0;  // (1: no fold work, 2: no release fence -- the timing experiments of r4_flash_gqa_fold_probe)
  }();
  // RoPE backward of dQ in the dQ kernel's epilogue (deterministic mode, GQA partials to fold; the
  // direct no-GQA path rotates Q and K in one rope_bwd_ pass)
  // (no GQA: the dK rotation too happens in the dK/dV kernel's store, so no rope_bwd_ pass follows;
  // flash_set_direct_rope(false) restores that pass, for A/B)
  const bool krot = rope && direct && g_direct_rope;
  const bool q_rot = rope && det && (!direct || krot);
  const float* dq_cos = q_rot ? cptr<float>(*cos_t) : nullptr;
  const float* dq_sin = q_rot ? cptr<float>(*sin_t) : nullptr;
  GqaFold fold{nullptr, mptr<bf16_t>(dqkv), rope ? cptr<float>(*cos_t) : nullptr,
               rope ? cptr<float>(*sin_t) : nullptr, fold_dbg, q_rot ? 1 : 0, krot ? 1 : 0};
  // the in-kernel fold holds at most 8 q-head partials per unit (uint4 x[U][8]): wider groups
  // take the finalize pass
  if (use_dkdv2 && !direct && g_bwd_fold && Hq / Hkv <= 8)
    fold.cnt = fold_counters(qk.device(), (long)B * Hkv * ((S + 32 * nw_ - 1) / (32 * nw_)));
  // 3-kernel GQA backward (g_fold3): dK/dV first (delta from O), then dQ + the fold; a column slice
  // of D / G columns per q-head block must be whole 16-B chunks
  const bool fold3 = use_dkdv2 && !direct && g_fold3 && fold.cnt == nullptr && D % (8 * (Hq / Hkv)) == 0;
  const bf16_t* fkp = fold3 ? dkp : nullptr;
  const bf16_t* fvp = fold3 ? dvp : nullptr;
  const int pre_blocks = (int)((rows * 16 + 255) / 256);
  const int nkt = (S + 127) / 128;
  dim3 grid(nkt * B * Hq), block(256);
  const int nw = nw_;
  const int nkt2 = (S + 32 * nw - 1) / (32 * nw);  // tiles of the deterministic dK/dV and dQ kernels
  const dim3 grid2(nkt2 * B * Hq), block2(64 * nw);
  float* dqp = det ? nullptr : mptr<float>(dq_acc);
#define FT_BWD(DD, MODE)                                                                          \
  hipLaunchKernelGGL((flash_bwd_kernel<E, DD, MODE>), grid, block, 0, ft_stream(), cptr<bf16_t>(dout), \
                     cptr<bf16_t>(qk), cptr<bf16_t>(qkv), cptr<float>(lse), cptr<float>(delta),     \
                     dqp, dkp, dvp, B, (int)S, (int)Hq, (int)Hkv,                                    \
                     sl2, scale, ldqk)
  // dK/dV split, head_dim 64 only (at 128 the doubled block spills): FT_FLASH_KV_SPLIT=0/1
  // forces; default: grids of at most one wave per SIMD
  const bool kv_split = D == 64 && (g_kv_split >= 0 ? g_kv_split == 1 : (long)grid2.x * nw <= 1024);
#define FT_DKDV2(DD, NW_, SP_)                                                                             \
  if (fold3)                                                                                                 \
    hipLaunchKernelGGL((flash_bwd_dkdv2_kernel<E, DD, NW_, SP_, true>), grid2, dim3(64 * NW_ * SP_), 0,        \
                       ft_stream(), cptr<bf16_t>(dout), cptr<bf16_t>(qk), cptr<bf16_t>(qkv), cptr<float>(lse), \
                       cptr<float>(delta), dkp, dvp, ldkv, B, (int)S, (int)Hq, (int)Hkv, sl2, scale, ldqk, fold, \
                       cptr<bf16_t>(out));                                                                   \
  else                                                                                                       \
    hipLaunchKernelGGL((flash_bwd_dkdv2_kernel<E, DD, NW_, SP_>), grid2, dim3(64 * NW_ * SP_), 0, ft_stream(), \
                       cptr<bf16_t>(dout), cptr<bf16_t>(qk), cptr<bf16_t>(qkv), cptr<float>(lse),         \
                       cptr<float>(delta), dkp, dvp, ldkv, B, (int)S,                                     \
                       (int)Hq, (int)Hkv, sl2, scale, ldqk, fold, nullptr)
  // dQ key split by default (FT_FLASH_DQ_SPLIT=0 turns it off): S = 2048, 12 heads of 64:
  // 94 -> 83 us for the whole backward; 8B layer 173 -> 167 us; S = 16384 1006 -> 972 us
  // (profiles/r2_flash_key_split.log)
  const bool dq_split = g_dq_split != 0;
  // deterministic mode: the dQ kernel runs first and forms delta itself (no flash_bwd_pre pass),
  // then the dK / dV kernel reads it
#define FT_DQ(DD, NW_)                                                                                  \
  if (dq_split)                                                                                         \
    hipLaunchKernelGGL((flash_bwd_dq_kernel<E, DD, NW_, 2>), grid2, dim3(128 * NW_), 0, ft_stream(),       \
                       cptr<bf16_t>(dout), cptr<bf16_t>(qk), cptr<bf16_t>(qkv), cptr<float>(lse),       \
                       mptr<float>(delta), mptr<bf16_t>(dqkv), B, (int)S, (int)Hq, (int)Hkv, sl2, scale, ldqk, \
                       cptr<bf16_t>(out), dq_cos, dq_sin, fkp, fvp);                                    \
  else                                                                                                  \
    hipLaunchKernelGGL((flash_bwd_dq_kernel<E, DD, NW_, 1>), grid2, block2, 0, ft_stream(),                \
                       cptr<bf16_t>(dout), cptr<bf16_t>(qk), cptr<bf16_t>(qkv), cptr<float>(lse),       \
                       mptr<float>(delta), mptr<bf16_t>(dqkv), B, (int)S, (int)Hq, (int)Hkv, sl2, scale, ldqk, \
                       cptr<bf16_t>(out), dq_cos, dq_sin, fkp, fvp)
  // the two deterministic kernels in their order: dQ first (it forms delta for the dK/dV kernel), or
  // -- fold3 -- dK/dV first (forms delta itself) and dQ after it (folds the partials it wrote)
#define FT_PAIR(DQ_STMT, KV_STMT) \
  if (fold3) {                    \
    KV_STMT;                      \
    DQ_STMT;                      \
  } else {                        \
    DQ_STMT;                      \
    KV_STMT;                      \
  }
#define FT_PRE(DD)                                                                                      \
  hipLaunchKernelGGL((flash_bwd_pre_kernel<E, DD>), dim3(pre_blocks), block, 0, ft_stream(),             \
                     cptr<bf16_t>(dout), cptr<bf16_t>(out), mptr<float>(delta), B, (int)S, (int)Hq)
  FT_DISPATCH_E16(qk.scalar_type(), {
    if (D == 128) {
      if (mode == 0) { FT_PRE(128); FT_BWD(128, 0); }
      else if (mode == 1) {
        if (g_dkdv2 && nw == 4) { FT_PAIR({ FT_DQ(128, 4); }, { FT_DKDV2(128, 4, 1); }) }
        else { FT_DQ(128, 4); FT_BWD(128, 1); }
      }
      else { FT_PRE(128); FT_BWD(128, 2); }
    } else {
      if (mode == 0) { FT_PRE(64); FT_BWD(64, 0); }
      else if (mode == 1 && nw == 2) {
        if (kv_split) { FT_PAIR({ FT_DQ(64, 2); }, { FT_DKDV2(64, 2, 2); }) }
        else { FT_PAIR({ FT_DQ(64, 2); }, { FT_DKDV2(64, 2, 1); }) }
      }
      // head_dim 64 with 4-wave blocks: the one-slice dK/dV kernel is faster (S = 8192, 16 heads:
      // 631 vs 783 us, profiles/r2_flash_long_context.log); FT_FLASH_DKDV2=2 forces the slice pair
      else if (mode == 1) {
        if (g_dkdv2_64 && kv_split) { FT_PAIR({ FT_DQ(64, 4); }, { FT_DKDV2(64, 4, 2); }) }
        else if (g_dkdv2_64) { FT_PAIR({ FT_DQ(64, 4); }, { FT_DKDV2(64, 4, 1); }) }
        else { FT_DQ(64, 4); FT_BWD(64, 1); }
      }
      else { FT_PRE(64); FT_BWD(64, 2); }
    }
  });
#undef FT_BWD
#undef FT_DKDV2
#undef FT_DQ
#undef FT_PAIR
#undef FT_PRE
  FT_LAUNCH_CHECK();
  if (direct) {  // no GQA partials to fold: only the RoPE backward remains (unless done in-kernel)
    if (rope && !krot) rope_bwd_(dqkv, *cos_t, *sin_t, S, Hq, Hkv, D);
    return dqkv;
  }
  if (fold.cnt != nullptr) return dqkv;  // folded by the dK/dV kernel's last block per tile
  if (fold3) return dqkv;                // folded by the dQ kernel
  const long vec = (long)T * ((Hq + 2 * Hkv) * D / 4);
  const int fin_blocks = (int)std::max(1L, std::min((vec + 255) / 256, 4096L));
  FT_DISPATCH_E16(qk.scalar_type(),
                  hipLaunchKernelGGL((flash_bwd_finalize_kernel<E>), dim3(fin_blocks), block, 0, ft_stream(),
                                     det ? nullptr : cptr<float>(dq_acc), cptr<bf16_t>(dk_part),
                                     cptr<bf16_t>(dv_part), mptr<bf16_t>(dqkv), (long)T, (int)Hq,
                                     (int)Hkv, (int)D, rope ? cptr<float>(*cos_t) : nullptr,
                                     rope ? cptr<float>(*sin_t) : nullptr, (int)S, q_rot ? 1 : 0));
  FT_LAUNCH_CHECK();
  return dqkv;
}

// Same-process A/B switch: slice-pair dK/dV kernel vs flash_bwd_kernel<D, 1>.
void flash_set_dkdv2(bool on) { g_dkdv2 = on; }
// Same-process A/B switch of the forward key split: -1 auto, 0 off, 1 on.
void flash_set_fwd_split(int64_t v) { g_fwd_split = (int)v; }
void flash_set_dq_split(int64_t v) { g_dq_split = (int)v; }
void flash_set_fwd_pipe(int64_t v) { g_fwd_pipe = (int)v; }
void flash_set_fwd_prof(const std::optional<at::Tensor>& buf) {
  if (buf.has_value()) {
    TORCH_CHECK(buf->scalar_type() == at::kLong && buf->is_contiguous(), "flash_set_fwd_prof: int64 buffer");
    g_fwd_prof = reinterpret_cast<long long*>(buf->data_ptr<int64_t>());
    g_fwd_prof_rows = buf->numel() / 8;
  } else {
    g_fwd_prof = nullptr;
    g_fwd_prof_rows = 0;
  }
}
void flash_set_kv_split(int64_t v) { g_kv_split = (int)v; }
void flash_set_bwd_fold(bool on) { g_bwd_fold = on; }
void flash_set_direct_rope(bool on) { g_direct_rope = on; }
void flash_set_fold3(bool on) { g_fold3 = on; }

TORCH_LIBRARY_FRAGMENT(ftamd, m) {
  m.def("flash_set_dkdv2(bool on) -> ()", &flash_set_dkdv2);
  m.def("flash_set_fwd_split(int v) -> ()", &flash_set_fwd_split);
  m.def("flash_set_dq_split(int v) -> ()", &flash_set_dq_split);
  m.def("flash_set_fwd_pipe(int v) -> ()", &flash_set_fwd_pipe);
  m.def("flash_set_fwd_prof(Tensor? buf) -> ()", &flash_set_fwd_prof);
  m.def("flash_set_kv_split(int v) -> ()", &flash_set_kv_split);
  m.def("flash_set_bwd_fold(bool on) -> ()", &flash_set_bwd_fold);
  m.def("flash_set_direct_rope(bool on) -> ()", &flash_set_direct_rope);
  m.def("flash_set_fold3(bool on) -> ()", &flash_set_fold3);
  m.def("flash_fwd(Tensor qk, Tensor qkv, int S, int Hq, int Hkv, int D) -> (Tensor, Tensor)",
        &flash_fwd);
  m.def(
      "flash_bwd(Tensor dout, Tensor qk, Tensor qkv, Tensor out, Tensor lse, int S, int Hq, int "
      "Hkv, int D, int mode=0, Tensor? cos=None, Tensor? sin=None) -> Tensor",
      &flash_bwd);
}
