// Hand-written bf16 GEMM for gfx950 (CDNA4): every layout the transformer step needs, one
// kernel family, fp32 accumulation on MFMA, fused epilogues.
//
//   C[M, N] (=|+=) sum_k A(m, k) * B(k, n)        bf16 in, fp32 accumulate, bf16 out
//
// Operand layouts (row-major storage, leading dimensions lda/ldb):
//   A_K  A(m, k) = a[m * lda + k]   (activations [T, K]; dY [T, N] of a dX GEMM)
//   A_M  A(m, k) = a[k * lda + m]   (dY^T of a weight-gradient GEMM: dY is [T, N], m = n)
//   B_K  B(k, n) = b[n * ldb + k]   (nn.Linear weight [N, K]: the forward)
//   B_N  B(k, n) = b[k * ldb + n]   (weight [N, K] read as K x N in dX; X [T, K] in dW)
// so the forward (A_K, B_K), dX (A_K, B_N) and dW (A_M, B_N) read the row-major
// activations and weights in place: no transpose kernel, no extra HBM pass (the
// hipBLASLt path needed 66 transposes per Llama-3-8B step for its preferred layout).
//
// Tiling (MI355X: 256 CUs, 160 KiB LDS, 64-wide waves, 4 SIMDs per CU):
//   256 x 256 output tile per 512-thread workgroup (8 waves as 2 (M) x 4 (N)), each
//   wave 128 x 64 = 8 x 4 fragments of v_mfma_f32_16x16x32_bf16 (128 fp32 acc VGPRs);
//   BK = 64, two LDS stages of A and B (128 KiB), filled by LDS-DMA
//   (global_load_lds_dwordx4: 16 B per lane straight into LDS, no staging VGPRs).
//   K-contiguous operands live in LDS as [256][64] with 16-B chunks XOR-swizzled by
//   row&7 (ds_read_b128 fragment reads conflict-free); M/N-contiguous operands as
//   [64][256] with 16-B units XOR-swizzled by 2*(k&3 | (k>>3&1)<<2), read with
//   ds_read_b64_tr_b16 (the hardware transpose delivers the k-major fragment;
//   conflict-free). The swizzle is applied to the DMA's per-lane SOURCE address
//   (the DMA destination is lane-linear), cdna_hip_programming.md rule 21.
//   The MFMA is issued with the B fragment as its A operand (D = B^T A^T = C^T), so
//   each lane ends with 4 consecutive output COLUMNS of one row: 8-byte stores.
// Work distribution: tiles are remapped XCD-contiguously (blockIdx % 8 selects the
// XCD) and rastered M-fastest inside an XCD's range, so neighbouring workgroups on one
// L2 share the B panel. Split-K (grid.z) writes fp32 slabs that a second kernel
// reduces and passes through the same epilogue; used when the tile count alone
// cannot fill the 256 CUs (M = 2048 tokens x N = 4096 is only 128 tiles).
//
// Epilogues: store; add a bf16 residual / accumulate into C (gradient accumulation,
// the residual stream of wo / w2); SwiGLU (gate/up columns interleaved per wave so
// a lane holds g and u of the same feature, writing silu(g)*u and the pre-activation);
// SwiGLU backward (dY of the activation in, dgate/dup out, pre-activation read back).
#include "torch_utils.h"

#include <utility>

namespace {

typedef __attribute__((address_space(3))) bf16x4_t lds_bf16x4_t;

template <typename F, int... I>
__device__ __forceinline__ void static_for_impl(F&& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  static_for_impl(f, std::make_integer_sequence<int, N>{});
}

constexpr int BM = 256, BN = 256, BK = 64, NT = 512;
constexpr int OP_BYTES = 256 * BK * 2;       // one operand tile per stage: 32 KiB
constexpr int STAGE_BYTES = 2 * OP_BYTES;    // A + B
constexpr int LDS_BYTES = 2 * STAGE_BYTES;   // two stages: 128 KiB

enum Epi : int {
  EPI_STORE = 0,    // C = acc                       (+ residual R if given)
  EPI_F32 = 1,      // fp32 split-K slab
  EPI_SWIGLU = 2,   // a = silu(g) * u, gu = [g | u]  (B rows interleaved by wave, see below)
  EPI_SWIGLU_BWD = 3,  // da in acc; dg, du from the saved gu
};

__device__ __forceinline__ void glds16(const void* g, char* lds_base) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                   (__attribute__((address_space(3))) void*)lds_base, 16, 0, 0);
}

__device__ __forceinline__ bf16x4_t ds_tr(const char* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4_t*)(p));
}

// swizzle of the [64][256] M/N-contiguous image: 16-B unit u of k-row k lives at u ^ swz(k)
__device__ __forceinline__ int swz_mn(int k) { return 2 * ((k & 3) | (((k >> 3) & 1) << 2)); }

// ---- LDS-DMA staging of one operand tile (256 rows/cols x 64 k) ---------------------------
// Each of the 512 threads issues 4 DMAs of 16 B; a wave's DMA covers 1 KiB of LDS.
// KC (K-contiguous): rows of 128 B, LDS chunk c' of row r holds global chunk c' ^ (r & 7).
//   `src` points at element (row0, k0); rows `ld` elements apart.
// MN (M/N-contiguous): k-rows of 512 B, LDS unit u' of row k holds global unit u' ^ swz(k).
//   `src` points at element (k0, col0); k-rows `ld` elements apart.
template <bool KC>
__device__ __forceinline__ void stage_tile(const bf16_t* __restrict__ src, long ld, char* lds, int wid,
                                           int lane) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int blk = i * 8 + wid;  // 1 KiB block of the image
    const bf16_t* g;
    if constexpr (KC) {
      const int r = blk * 8 + (lane >> 3);
      const int c = (lane & 7) ^ (r & 7);
      g = src + (long)r * ld + c * 8;
    } else {
      const int k = blk * 2 + (lane >> 5);
      const int u = (lane & 31) ^ swz_mn(k);
      g = src + (long)k * ld + u * 8;
    }
    glds16(g, lds + blk * 1024);
  }
}

// ---- fragment reads (16 rows/cols x 32 k, the 16x16x32 operand map) ------------------------
// Lane l gets element j of (row r0 + (l & 15), k = kk*32 + 8*(l >> 4) + j).
template <bool KC>
__device__ __forceinline__ bf16x8_t frag(const char* img, int r0, int kk, int lane) {
  if constexpr (KC) {
    const int r = r0 + (lane & 15);
    const int c = kk * 4 + (lane >> 4);
    return *reinterpret_cast<const bf16x8_t*>(img + r * 128 + ((c ^ (r & 7)) << 4));
  } else {
    const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
    const int k = kk * 32 + 8 * g + q;
    const int u = (r0 >> 3) + (p >> 1);
    const int half = (p & 1) * 8;
    const bf16x4_t lo = ds_tr(img + k * 512 + ((u ^ swz_mn(k)) << 4) + half);
    const bf16x4_t hi = ds_tr(img + (k + 4) * 512 + ((u ^ swz_mn(k + 4)) << 4) + half);
    bf16x8_t r;
    r[0] = lo[0]; r[1] = lo[1]; r[2] = lo[2]; r[3] = lo[3];
    r[4] = hi[0]; r[5] = hi[1]; r[6] = hi[2]; r[7] = hi[3];
    return r;
  }
}

// The same fragment reads issued by inline asm (AR kernels: the one-barrier schedule of the
// dX / dW layouts). The compiler's waitcnt pass cannot tell a __builtin ds_read_tr (nor, next
// to it, a ds_read) from the LDS-DMA writes still in flight into the OTHER stage, so it put an
// s_waitcnt vmcnt(0) in front of the first fragment read of every K-tile: the DMA of tile t+2,
// issued a quarter-tile earlier, drained there, and the prefetch never overlapped more than
// one quarter of MFMAs. Reads the pass cannot see get no such wait; the loop waits for them
// with lgkm_wait<N>() (LDS reads return in order: N = reads issued after the ones needed).
__device__ __forceinline__ unsigned lds_addr(const char* p) {
  return (unsigned)(uintptr_t)((const __attribute__((address_space(3))) char*)p);
}

template <bool KC>
__device__ __forceinline__ bf16x8_t frag_asm(const char* img, int r0, int kk, int lane) {
  if constexpr (KC) {
    const int r = r0 + (lane & 15);
    const int c = kk * 4 + (lane >> 4);
    bf16x8_t v;
    asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(lds_addr(img + r * 128 + ((c ^ (r & 7)) << 4))) : "memory");
    return v;
  } else {
    const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
    const int k = kk * 32 + 8 * g + q;
    const int u = (r0 >> 3) + (p >> 1);
    const int half = (p & 1) * 8;
    bf16x4_t lo, hi;
    asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(lo) : "v"(lds_addr(img + k * 512 + ((u ^ swz_mn(k)) << 4) + half)) : "memory");
    asm volatile("ds_read_b64_tr_b16 %0, %1"
                 : "=v"(hi)
                 : "v"(lds_addr(img + (k + 4) * 512 + ((u ^ swz_mn(k + 4)) << 4) + half))
                 : "memory");
    bf16x8_t r;
    r[0] = lo[0]; r[1] = lo[1]; r[2] = lo[2]; r[3] = lo[3];
    r[4] = hi[0]; r[5] = hi[1]; r[6] = hi[2]; r[7] = hi[3];
    return r;
  }
}

template <int N>
__device__ __forceinline__ void lgkm_wait() {
  static_assert(N == 0 || N == 4 || N == 8 || N == 12 || N == 15, "lgkm_wait count");
  if constexpr (N == 0) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  else if constexpr (N == 4) asm volatile("s_waitcnt lgkmcnt(4)" ::: "memory");
  else if constexpr (N == 8) asm volatile("s_waitcnt lgkmcnt(8)" ::: "memory");
  else if constexpr (N == 12) asm volatile("s_waitcnt lgkmcnt(12)" ::: "memory");
  else asm volatile("s_waitcnt lgkmcnt(15)" ::: "memory");
}

// keeps the consumers of f after the preceding asm wait
__device__ __forceinline__ void tie(bf16x8_t (&f)[4]) {
#pragma unroll
  for (int i = 0; i < 4; ++i) asm volatile("" : "+v"(f[i]));
}

__device__ __forceinline__ float silu(float x) { return x / (1.f + __expf(-x)); }

struct GemmArgs {
  const bf16_t* a;
  const bf16_t* b;
  bf16_t* c;           // bf16 output (EPI_STORE / SWIGLU: a; SWIGLU_BWD: dgu)
  const bf16_t* r;     // residual added to the output (may alias c: accumulate); SWIGLU_BWD: gu
  bf16_t* c2;          // SWIGLU: gu output
  float* ws;           // EPI_F32: fp32 slabs [splits][M][N]
  long lda, ldb, ldc, ldr;
  int M, N, K;
  int k_per_split;
  int tiles_m, tiles_n;
  int ffn;             // SwiGLU: hidden size F (gate rows 0..F-1 of w13, up rows F..2F-1)
};

// Output tile for workgroup `bid`: XCD-contiguous ranges (bid % 8 = XCD under round-robin
// dispatch; bijective for any count), M-fastest raster inside a range.
__device__ __forceinline__ void tile_of(int bid, int tiles_m, int tiles_n, int& tm, int& tn) {
  const int nwg = tiles_m * tiles_n;
  const int q = nwg / 8, rem = nwg % 8;
  const int x = bid % 8, o = bid / 8;
  const int w = (x < rem ? x * (q + 1) : rem * (q + 1) + (x - rem) * q) + o;
  tm = w % tiles_m;
  tn = w / tiles_m;
}

// ABL (ablation builds for scripts/gemm_ablate.py only; 0 in every real launch):
// 1 no in-loop barrier/wait, 2 no in-loop DMA, 3 no in-loop LDS reads, 4 MFMAs only,
// 5 no wait for the DMAs before the barrier, 6 the one-barrier-per-tile schedule.
// (1-5 apply to the two-barrier schedule: the K-contiguous layouts)
// AR: fragment reads by inline asm with explicit lgkmcnt waits (one-barrier schedule only).
template <bool AK, bool BKC, int EPI, bool RES, int ABL = 0, bool AR = false>
__global__ __launch_bounds__(NT, 1) void gemm_kernel(GemmArgs p) {
  __shared__ __attribute__((aligned(1024))) char smem[LDS_BYTES];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid >> 2, wc = wid & 3;
  int tm, tn;
  tile_of(blockIdx.x, p.tiles_m, p.tiles_n, tm, tn);
  const int m0 = tm * BM, n0 = tn * BN;
  const int kz = blockIdx.y * p.k_per_split;
  const int nk = p.k_per_split / BK;

  // per-operand source of (tile, k0 = kz): advanced by BK each K-tile
  const bf16_t* a_src;
  long a_step;
  if constexpr (AK) {
    a_src = p.a + (long)m0 * p.lda + kz;
    a_step = BK;
  } else {
    a_src = p.a + (long)kz * p.lda + m0;
    a_step = (long)BK * p.lda;
  }
  // SwiGLU: B-tile column j of wave w' = j / 64 maps to gate feature (j % 32) of block
  // w' (j % 64 < 32) or to the matching up feature: a lane then holds g and u of one
  // feature in n-fragments f and f + 2. The 256-column tile covers 128 features.
  const bf16_t* b_src[2];
  long b_step;
  if constexpr (BKC) {
    if constexpr (EPI == EPI_SWIGLU) {
      // rows of w13 for this tile: gate rows fbase + [0,128), up rows F + fbase + [0,128);
      // staged as 256 LDS rows in the interleaved order (handled in the staging below)
      b_src[0] = p.b + (long)(tn * 128) * p.ldb + kz;
      b_src[1] = p.b + (long)(p.ffn + tn * 128) * p.ldb + kz;
    } else {
      b_src[0] = p.b + (long)n0 * p.ldb + kz;
      b_src[1] = nullptr;
    }
    b_step = BK;
  } else {
    b_src[0] = p.b + (long)kz * p.ldb + n0;
    b_src[1] = nullptr;
    b_step = (long)BK * p.ldb;
  }

  auto stage_a = [&](int t, int buf) {
    stage_tile<AK>(a_src + t * a_step, p.lda, smem + buf * STAGE_BYTES, wid, lane);
  };
  auto stage_b = [&](int t, int buf) {
    char* base = smem + buf * STAGE_BYTES + OP_BYTES;
    if constexpr (EPI == EPI_SWIGLU) {
      // interleaved rows: LDS row j <- gate/up feature as described above
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int blk = i * 8 + wid;
        const int r = blk * 8 + (lane >> 3);          // LDS row 0..255
        const int c = (lane & 7) ^ (r & 7);
        const int feat = (r >> 6) * 32 + (r & 31);    // feature within the tile's 128
        const bf16_t* src = b_src[(r >> 5) & 1] + t * b_step + (long)feat * p.ldb + c * 8;
        glds16(src, base + blk * 1024);
      }
    } else {
      stage_tile<BKC>(b_src[0] + t * b_step, p.ldb, base, wid, lane);
    }
  };
  auto stage = [&](int t, int buf) {
    stage_a(t, buf);
    stage_b(t, buf);
  };

  f32x4_t acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  // K-tile = 4 quarters of 16 MFMAs (4 m-fragments x 4 n-fragments, one 32-deep k-step):
  //   Q1 (kk 0, m 0-3) Q2 (kk 0, m 4-7) Q3 (kk 1, m 0-3) Q4 (kk 1, m 4-7).
  // The LDS reads of the next quarter's fragments are in flight while a quarter's MFMAs run
  // (two alternating register sets for A and for B: 64 VGPRs of operands beside the 128
  // accumulators). One barrier per K-tile, before Q4: by then every wave has read all of
  // tile t (A of Q4 was read during Q3) and its DMAs of tile t+1 have landed, so Q4's
  // MFMAs issue right after it while tile t+1's first fragments are read and the DMA of
  // tile t+2 overwrites tile t's buffer. Each DMA has a whole K-tile (Q4..Q3) to land.
  bf16x8_t aX[4], aY[4], bX[4], bY[4];
  auto read_a = [&](const char* st, int kk, int mh, bf16x8_t(&af)[4]) {
    static_for<4>([&](auto I) {
      if constexpr (AR)
        af[I] = frag_asm<AK>(st, wr * 128 + (mh * 4 + I) * 16, kk, lane);
      else
        af[I] = frag<AK>(st, wr * 128 + (mh * 4 + I) * 16, kk, lane);
    });
  };
  auto read_b = [&](const char* st, int kk, bf16x8_t(&bf)[4]) {
    static_for<4>([&](auto J) {
      if constexpr (AR)
        bf[J] = frag_asm<BKC>(st + OP_BYTES, wc * 64 + J * 16, kk, lane);
      else
        bf[J] = frag<BKC>(st + OP_BYTES, wc * 64 + J * 16, kk, lane);
    });
  };
  // AR: LDS read instructions per read_a / read_b (a transposed fragment is two reads)
  constexpr int RA = AK ? 4 : 8, RB = BKC ? 4 : 8;
  constexpr int RAB = RA + RB > 15 ? 15 : RA + RB;
  auto mma = [&](bf16x8_t(&af)[4], auto MH, bf16x8_t(&bf)[4]) {
    static_for<4>([&](auto I) {
      static_for<4>([&](auto J) {
        acc[MH * 4 + I][J] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[J], af[I], acc[MH * 4 + I][J], 0, 0, 0);
      });
    });
  };
  constexpr std::integral_constant<int, 0> H0{};
  constexpr std::integral_constant<int, 1> H1{};

  stage(0, 0);
  asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
  if (nk > 1) stage(1, 1);
  read_a(smem, 0, 0, aX);
  read_b(smem, 0, bX);
  constexpr bool RD = ABL != 3 && ABL != 4, DMA = ABL != 2 && ABL != 4, BAR = ABL != 1 && ABL != 4;
  if constexpr (!RD) {
    read_a(smem, 0, 1, aY);
    read_b(smem, 1, bY);
  }
  // Schedule per layout (scripts/gemm_ablate.py, scripts/gemm_bench.py on MI355X): the
  // two-barrier schedule below wins for the all-K-contiguous forward (+7..25 %); with a
  // transposed-read operand (24 tr-read addresses live) it loses 10-20 %, so dX / dW keep
  // one barrier per K-tile with all DMAs of tile t+2 in Q4.
  constexpr bool ONE_BAR = ABL == 6 || !(AK && BKC);
  static_assert(!AR || ONE_BAR, "asm reads: one-barrier schedule only");
  if constexpr (ONE_BAR) {
    for (int t = 0; t < nk; ++t) {
      const char* cur = smem + (t & 1) * STAGE_BYTES;
      read_a(cur, 0, 1, aY);
      if constexpr (AR) {  // aX, bX landed; aY may be in flight
        lgkm_wait<RA>();
        tie(aX);
        tie(bX);
      }
      mma(aX, H0, bX);
      read_a(cur, 1, 0, aX);
      read_b(cur, 1, bY);
      if constexpr (AR) {  // aY landed
        lgkm_wait<RAB>();
        tie(aY);
      }
      mma(aY, H1, bX);
      read_a(cur, 1, 1, aY);
      if constexpr (AR) {  // aX, bY landed
        lgkm_wait<RA>();
        tie(aX);
        tie(bY);
      }
      mma(aX, H0, bY);
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
      if constexpr (AR) {  // aY (and bY) landed at the barrier's wait
        tie(aY);
        tie(bY);
      }
      if (t + 1 < nk) {
        const char* nxt = smem + ((t + 1) & 1) * STAGE_BYTES;
        read_a(nxt, 0, 0, aX);
        read_b(nxt, 0, bX);
      }
      if (t + 2 < nk) stage(t + 2, t & 1);
      mma(aY, H1, bY);
    }
  } else {
    // Two barriers per K-tile. X (after Q2): every wave has read all of B(t) -> Q3 DMAs
    // B(t+2) into that buffer. Y (after Q3): all of A(t) read, and tile t+1 landed (its A
    // went out in Q4(t-1), its B in Q3(t-1): vmcnt(4) leaves B(t+2) in flight) -> Q4
    // DMAs A(t+2) and reads tile t+1's first fragments. The DMA issue is spread over two
    // quarters and B gets five quarters to land, A four.
    for (int t = 0; t < nk; ++t) {
      const char* cur = smem + (t & 1) * STAGE_BYTES;
      if constexpr (RD) read_a(cur, 0, 1, aY);   // Q1
      mma(aX, H0, bX);
      if constexpr (RD) {                         // Q2
        read_a(cur, 1, 0, aX);
        read_b(cur, 1, bY);
      }
      mma(aY, H1, bX);
      if constexpr (BAR) asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // X
      if (DMA && t + 2 < nk) stage_b(t + 2, t & 1);                                       // Q3
      if constexpr (RD) read_a(cur, 1, 1, aY);
      mma(aX, H0, bY);
      if constexpr (ABL == 5) {
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      } else if constexpr (BAR) {                                                          // Y
        if (t + 2 < nk)
          asm volatile("s_waitcnt vmcnt(4) lgkmcnt(0)\n\ts_barrier" ::: "memory");
        else
          asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
      }
      if (DMA && t + 2 < nk) stage_a(t + 2, t & 1);                                       // Q4
      if (RD && t + 1 < nk) {
        const char* nxt = smem + ((t + 1) & 1) * STAGE_BYTES;
        read_a(nxt, 0, 0, aX);
        read_b(nxt, 0, bX);
      }
      mma(aY, H1, bY);
    }
  }
  if constexpr (!RD || !DMA) asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");

  // ---- epilogue: lane holds rows m = .. + (lane & 15), columns n = .. + 4*(lane >> 4) + r
  const int lr = lane & 15, lc = (lane >> 4) * 4;
  constexpr bool has_r = RES;
  if constexpr (EPI == EPI_F32) {
    float* ws = p.ws + (long)blockIdx.y * p.M * p.N;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int m = m0 + wr * 128 + i * 16 + lr;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int n = n0 + wc * 64 + j * 16 + lc;
        *reinterpret_cast<f32x4_t*>(ws + (long)m * p.N + n) = acc[i][j];
      }
    }
  } else if constexpr (EPI == EPI_SWIGLU) {
    // n-fragments 0,1: gate of features wc*32 + [0,32); 2,3: up of the same features
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int m = m0 + wr * 128 + i * 16 + lr;
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int f = tn * 128 + wc * 32 + j * 16 + lc;  // feature index
        const f32x4_t g = acc[i][j], u = acc[i][j + 2];
        uint2 ov, gv, uv;
        // g, u are rounded to bf16 (the saved pre-activation, as the unfused GEMM output);
        // the activation in fp32 with one rounding, as swiglu.hip
        float gr[4], ur[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          gr[r] = bf2f(f2bf(g[r]));
          ur[r] = bf2f(f2bf(u[r]));
        }
        ov.x = pack2(silu(gr[0]) * ur[0], silu(gr[1]) * ur[1]);
        ov.y = pack2(silu(gr[2]) * ur[2], silu(gr[3]) * ur[3]);
        gv.x = pack2(gr[0], gr[1]);
        gv.y = pack2(gr[2], gr[3]);
        uv.x = pack2(ur[0], ur[1]);
        uv.y = pack2(ur[2], ur[3]);
        *reinterpret_cast<uint2*>(p.c + (long)m * p.ldc + f) = ov;
        *reinterpret_cast<uint2*>(p.c2 + (long)m * (2L * p.ffn) + f) = gv;
        *reinterpret_cast<uint2*>(p.c2 + (long)m * (2L * p.ffn) + p.ffn + f) = uv;
      }
    }
  } else {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int m = m0 + wr * 128 + i * 16 + lr;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int n = n0 + wc * 64 + j * 16 + lc;
        f32x4_t v = acc[i][j];
        if constexpr (EPI == EPI_SWIGLU_BWD) {
          // acc = da for features n..n+3; gu holds g at [m][n], u at [m][F + n]
          const uint2 gv = *reinterpret_cast<const uint2*>(p.r + (long)m * p.ldr + n);
          const uint2 uv = *reinterpret_cast<const uint2*>(p.r + (long)m * p.ldr + p.ffn + n);
          float g[4] = {__uint_as_float(gv.x << 16), __uint_as_float(gv.x & 0xffff0000u),
                        __uint_as_float(gv.y << 16), __uint_as_float(gv.y & 0xffff0000u)};
          float u[4] = {__uint_as_float(uv.x << 16), __uint_as_float(uv.x & 0xffff0000u),
                        __uint_as_float(uv.y << 16), __uint_as_float(uv.y & 0xffff0000u)};
          float dg[4], du[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float da = bf2f(f2bf(v[r]));  // da is a bf16 GEMM output in the unfused path
            const float sg = 1.f / (1.f + __expf(-g[r]));
            const float sl = g[r] * sg;
            du[r] = da * sl;
            dg[r] = da * u[r] * (sg + sl * (1.f - sg));  // same math as swiglu.hip
          }
          uint2 o1, o2;
          o1.x = pack2(dg[0], dg[1]);
          o1.y = pack2(dg[2], dg[3]);
          o2.x = pack2(du[0], du[1]);
          o2.y = pack2(du[2], du[3]);
          *reinterpret_cast<uint2*>(p.c + (long)m * p.ldc + n) = o1;
          *reinterpret_cast<uint2*>(p.c + (long)m * p.ldc + p.ffn + n) = o2;
        } else {
          if (has_r) {
            const uint2 rv = *reinterpret_cast<const uint2*>(p.r + (long)m * p.ldr + n);
            v[0] += __uint_as_float(rv.x << 16);
            v[1] += __uint_as_float(rv.x & 0xffff0000u);
            v[2] += __uint_as_float(rv.y << 16);
            v[3] += __uint_as_float(rv.y & 0xffff0000u);
          }
          uint2 o;
          o.x = pack2(v[0], v[1]);
          o.y = pack2(v[2], v[3]);
          *reinterpret_cast<uint2*>(p.c + (long)m * p.ldc + n) = o;
        }
      }
    }
  }
}

// ---- 128 x 128 tiles: the small-model GEMMs ---------------------------------------------------
// Products with fewer than 128 output tiles of 256 x 256 (GPT-2-class d = 768 / 1024 at
// T = 2048: 24-96 tiles) or M / N not multiples of 256. A 256-thread workgroup (4 waves,
// 2 x 2, each 64 x 64 = 4 x 4 fragments, 64 fp32 acc VGPRs) owns a 128 x 128 tile, 4x the
// workgroups of the 256 kernel; two LDS stages of 32 KiB (A + B, BK = 64) filled by LDS-DMA,
// two workgroups per CU. One barrier per K-tile (see the loop). Tall K with few tiles splits
// K (pick_splits128). Same operand layouts, swizzles, fragment map and epilogues as the 256
// kernel; M/N-contiguous operand images are [64][128] (256-B k-rows: the swz_mn XOR stays in
// a row). Measured (profiles/r2_gemm_small_tiles.log): 1.4-2x the 256 kernel on those shapes
// but 0.6-1.0x hipBLASLt, so the default routing keeps hipBLASLt for them (ops/functional.py).
constexpr int S_T = 128, S_NT = 256;
constexpr int S_OP = S_T * BK * 2;  // 16 KiB
constexpr int S_STAGE = 2 * S_OP;

template <bool KC>
__device__ __forceinline__ void stage_tile128(const bf16_t* __restrict__ src, long ld, char* lds, int wid,
                                              int lane) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int blk = i * 4 + wid;  // 1 KiB block of the 16 KiB image
    const bf16_t* g;
    if constexpr (KC) {
      const int r = blk * 8 + (lane >> 3);
      const int c = (lane & 7) ^ (r & 7);
      g = src + (long)r * ld + c * 8;
    } else {
      const int k = blk * 4 + (lane >> 4);
      const int u = (lane & 15) ^ swz_mn(k);
      g = src + (long)k * ld + u * 8;
    }
    glds16(g, lds + blk * 1024);
  }
}

template <bool KC>
__device__ __forceinline__ bf16x8_t frag128(const char* img, int r0, int kk, int lane) {
  if constexpr (KC) {
    return frag<true>(img, r0, kk, lane);
  } else {
    const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
    const int k = kk * 32 + 8 * g + q;
    const int u = (r0 >> 3) + (p >> 1);
    const int half = (p & 1) * 8;
    const bf16x4_t lo = ds_tr(img + k * 256 + ((u ^ swz_mn(k)) << 4) + half);
    const bf16x4_t hi = ds_tr(img + (k + 4) * 256 + ((u ^ swz_mn(k + 4)) << 4) + half);
    bf16x8_t r;
    r[0] = lo[0]; r[1] = lo[1]; r[2] = lo[2]; r[3] = lo[3];
    r[4] = hi[0]; r[5] = hi[1]; r[6] = hi[2]; r[7] = hi[3];
    return r;
  }
}

template <bool AK, bool BKC, int EPI, bool RES>
__global__ __launch_bounds__(S_NT, 2) void gemm128_kernel(GemmArgs p) {
  constexpr int NS = 2;  // 3-4 stages (1 workgroup per CU) measured slower: profiles/r2_gemm_small_tiles.log
  __shared__ __attribute__((aligned(1024))) char smem[NS * S_STAGE];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid >> 1, wc = wid & 1;
  int tm, tn;
  tile_of(blockIdx.x, p.tiles_m, p.tiles_n, tm, tn);
  const int m0 = tm * S_T, n0 = tn * S_T;
  const int kz = blockIdx.y * p.k_per_split;
  const int nk = p.k_per_split / BK;

  const bf16_t* a_src = AK ? p.a + (long)m0 * p.lda + kz : p.a + (long)kz * p.lda + m0;
  const long a_step = AK ? (long)BK : (long)BK * p.lda;
  const bf16_t* b_src = BKC ? p.b + (long)n0 * p.ldb + kz : p.b + (long)kz * p.ldb + n0;
  const long b_step = BKC ? (long)BK : (long)BK * p.ldb;
  auto stage = [&](int t) {
    char* base = smem + (t % NS) * S_STAGE;
    stage_tile128<AK>(a_src + t * a_step, p.lda, base, wid, lane);
    stage_tile128<BKC>(b_src + t * b_step, p.ldb, base + S_OP, wid, lane);
  };

  f32x4_t acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  // X / Y: fragments of k-steps 0 / 1 of a K-tile. Y's LDS reads are in flight while X's 16
  // MFMAs run, the next tile's X reads while Y's run; the barrier between (after X) publishes
  // tile t + 1 and retires every wave's reads of tile t, whose buffer then takes tile t + NS.
  bf16x8_t xa[4], xb[4], ya[4], yb[4];
  auto rd = [&](const char* st, int kk, bf16x8_t(&fa)[4], bf16x8_t(&fb)[4]) {
    static_for<4>([&](auto I) { fa[I] = frag128<AK>(st, wr * 64 + I * 16, kk, lane); });
    static_for<4>([&](auto J) { fb[J] = frag128<BKC>(st + S_OP, wc * 64 + J * 16, kk, lane); });
  };
  auto mma = [&](bf16x8_t(&fa)[4], bf16x8_t(&fb)[4]) {
    static_for<4>([&](auto I) {
      static_for<4>([&](auto J) {
        acc[I][J] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[J], fa[I], acc[I][J], 0, 0, 0);
      });
    });
  };
#pragma unroll
  for (int t = 0; t < NS; ++t)
    if (t < nk) stage(t);
  if (nk > 1)
    asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  rd(smem, 0, xa, xb);
  for (int t = 0; t < nk; ++t) {
    const char* cur = smem + (t % NS) * S_STAGE;
    rd(cur, 1, ya, yb);
    mma(xa, xb);
    if (t + 1 < nk) {
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");  // tile t + 1 landed
      if (t + NS < nk) stage(t + NS);
      rd(smem + ((t + 1) % NS) * S_STAGE, 0, xa, xb);
    }
    mma(ya, yb);
  }

  const int lr = lane & 15, lc = (lane >> 4) * 4;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = m0 + wr * 64 + i * 16 + lr;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int n = n0 + wc * 64 + j * 16 + lc;
      f32x4_t v = acc[i][j];
      if constexpr (EPI == EPI_F32) {
        *reinterpret_cast<f32x4_t*>(p.ws + (long)blockIdx.y * p.M * p.N + (long)m * p.N + n) = v;
      } else {
        if constexpr (RES) {
          const uint2 rv = *reinterpret_cast<const uint2*>(p.r + (long)m * p.ldr + n);
          v[0] += __uint_as_float(rv.x << 16);
          v[1] += __uint_as_float(rv.x & 0xffff0000u);
          v[2] += __uint_as_float(rv.y << 16);
          v[3] += __uint_as_float(rv.y & 0xffff0000u);
        }
        uint2 o;
        o.x = pack2(v[0], v[1]);
        o.y = pack2(v[2], v[3]);
        *reinterpret_cast<uint2*>(p.c + (long)m * p.ldc + n) = o;
      }
    }
  }
}

// Split-K reduction: out = sum_z ws[z] (+ residual), bf16; 8 outputs per thread.
__global__ __launch_bounds__(256) void splitk_reduce_kernel(const float* __restrict__ ws, int splits,
                                                            long MN, int N, bf16_t* __restrict__ c, long ldc,
                                                            const bf16_t* __restrict__ r, long ldr) {
  const long i8 = (long)blockIdx.x * 256 + threadIdx.x;
  const long e = i8 * 8;
  if (e >= MN) return;
  float v[8];
  {
    const float4 a = *reinterpret_cast<const float4*>(ws + e);
    const float4 b = *reinterpret_cast<const float4*>(ws + e + 4);
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
  }
  for (int z = 1; z < splits; ++z) {
    const float4 a = *reinterpret_cast<const float4*>(ws + z * MN + e);
    const float4 b = *reinterpret_cast<const float4*>(ws + z * MN + e + 4);
    v[0] += a.x; v[1] += a.y; v[2] += a.z; v[3] += a.w; v[4] += b.x; v[5] += b.y; v[6] += b.z; v[7] += b.w;
  }
  const long m = e / N, n = e % N;
  if (r != nullptr) {
    float rf[8];
    unpack8(*reinterpret_cast<const uint4*>(r + m * ldr + n), rf);
#pragma unroll
    for (int q = 0; q < 8; ++q) v[q] += rf[q];
  }
  *reinterpret_cast<uint4*>(c + m * ldc + n) = pack8(v);
}

// Fragment reads by inline asm in the one-barrier (dX / dW layout) kernels: 1 (default) or 0
// (builtin reads; FT_GEMM_ASM_READS / gemm_config, for A/B). See frag_asm.
int g_asm_reads = [] {
  const char* e = std::getenv("FT_GEMM_ASM_READS");
  return e == nullptr ? 1 : std::atoi(e);
}();

template <bool AK, bool BKC, int EPI>
void launch(const GemmArgs& a, int splits, hipStream_t s) {
  const dim3 g(a.tiles_m * a.tiles_n, splits);
  // residual only matters for the bf16 store epilogue (split-K adds it in the reduction)
  const bool res = EPI == EPI_STORE && a.r != nullptr;
  if constexpr (!(AK && BKC)) {
    if (g_asm_reads) {
      if (res)
        hipLaunchKernelGGL((gemm_kernel<AK, BKC, EPI, true, 0, true>), g, dim3(NT), 0, s, a);
      else
        hipLaunchKernelGGL((gemm_kernel<AK, BKC, EPI, false, 0, true>), g, dim3(NT), 0, s, a);
      return;
    }
  }
  if (res)
    hipLaunchKernelGGL((gemm_kernel<AK, BKC, EPI, true>), g, dim3(NT), 0, s, a);
  else
    hipLaunchKernelGGL((gemm_kernel<AK, BKC, EPI, false>), g, dim3(NT), 0, s, a);
}

int g_tile = 0;     // 0: pick per shape; 128 / 256: force (scripts/gemm_bench.py A/B)
template <bool AK, bool BKC, int EPI>
void launch128(const GemmArgs& a, int splits, hipStream_t s) {
  const dim3 g(a.tiles_m * a.tiles_n, splits), b(S_NT);
  if (EPI == EPI_STORE && a.r != nullptr)
    hipLaunchKernelGGL((gemm128_kernel<AK, BKC, EPI, true>), g, b, 0, s, a);
  else
    hipLaunchKernelGGL((gemm128_kernel<AK, BKC, EPI, false>), g, b, 0, s, a);
}

// Splits so that tiles x splits reaches about the CU count (256) without slicing K below 1024;
// a tall-K product with few output tiles (GPT-2's LM-head dX: 24 tiles, K = 131072) goes to
// ~2 workgroups per CU, where the fp32 slabs are still small next to the GEMM.
int pick_splits(int tiles, int K) {
  int s = 1;
  const int target = tiles < 64 ? 400 : 200;
  while (tiles * s < target && (K / (s * 2)) % BK == 0 && K / (s * 2) >= 1024) s *= 2;
  return s;
}

// 128 tiles: split K (>= 512 per split) while the grid is under the CU count.
int pick_splits128(int tiles, int K) {
  int s = 1;
  while (tiles * s < 256 && (K / (s * 2)) % BK == 0 && K / (s * 2) >= 512) s *= 2;
  return s;
}

}  // namespace

// C = op(A) @ op(B) (+ R), bf16. Layout codes: a_kc: A is [M, K] (else A^T stored [K, M]);
// b_kc: B is given as [N, K] (else [K, N]). `out` may be given (written in place; with
// accumulate=True it is also added: out += A@B).
at::Tensor gemm(const at::Tensor& a, bool a_kc, const at::Tensor& b, bool b_kc, int64_t M, int64_t N, int64_t K,
                const std::optional<at::Tensor>& out, const std::optional<at::Tensor>& residual, bool accumulate,
                int64_t splits) {
  FT_CHECK_CUDA(a);
  FT_CHECK_BF16(a);
  FT_CHECK_BF16(b);
  FT_CHECK_CONTIG(a);
  FT_CHECK_CONTIG(b);
  TORCH_CHECK(M % S_T == 0 && N % S_T == 0 && K % BK == 0, "gemm: M, N must be multiples of 128 and K of 64 (got ",
              M, " ", N, " ", K, ")");
  // 256 x 256 tiles when they fill the chip (>= 128 tiles) or split-K over a tall K does;
  // 128 x 128 tiles otherwise (4x the workgroups)
  const bool fits256 = M % BM == 0 && N % BN == 0;
  const bool big = g_tile == 256 || (g_tile == 0 && fits256 && ((M / BM) * (N / BN) >= 128 || K >= 16384));
  TORCH_CHECK(!big || fits256, "gemm: 256 tiles need M, N multiples of 256");
  TORCH_CHECK(a.numel() == M * K && b.numel() == N * K, "gemm: operand sizes do not match M, N, K");
  const at::DeviceGuard guard(a.device());
  at::Tensor c;
  if (out.has_value() && out->defined()) {
    c = *out;
    FT_CHECK_BF16(c);
    FT_CHECK_CONTIG(c);
    TORCH_CHECK(c.numel() == M * N, "gemm: out has the wrong size");
  } else {
    TORCH_CHECK(!accumulate, "gemm: accumulate needs out");
    c = at::empty({M, N}, a.options());
  }
  const bf16_t* rp = nullptr;
  if (accumulate) {
    rp = cptr<bf16_t>(c);
  } else if (residual.has_value() && residual->defined()) {
    FT_CHECK_BF16((*residual));
    FT_CHECK_CONTIG((*residual));
    TORCH_CHECK(residual->numel() == M * N, "gemm: residual has the wrong size");
    rp = cptr<bf16_t>(*residual);
  }
  GemmArgs p{};
  p.a = cptr<bf16_t>(a);
  p.b = cptr<bf16_t>(b);
  p.c = mptr<bf16_t>(c);
  p.r = rp;
  p.lda = a_kc ? K : M;
  p.ldb = b_kc ? K : N;
  p.ldc = N;
  p.ldr = N;
  p.M = M;
  p.N = N;
  p.K = K;
  const int tile = big ? BM : S_T;
  p.tiles_m = M / tile;
  p.tiles_n = N / tile;
  int s = splits > 0 ? (int)splits : (big ? pick_splits(p.tiles_m * p.tiles_n, K) : pick_splits128(p.tiles_m * p.tiles_n, K));
  TORCH_CHECK(K % (s * BK) == 0, "gemm: K must split into multiples of 64");
  p.k_per_split = K / s;
  hipStream_t st = ft_stream();
  at::Tensor ws;
  if (s > 1) {
    ws = at::empty({s, M, N}, a.options().dtype(at::kFloat));
    p.ws = mptr<float>(ws);
  }
#define FT_GEMM_LAUNCH(AK_, BK_)                                                             \
  if (!big && s > 1)                                                                         \
    launch128<AK_, BK_, EPI_F32>(p, s, st);                                                  \
  else if (!big)                                                                             \
    launch128<AK_, BK_, EPI_STORE>(p, s, st);                                                \
  else if (s > 1)                                                                            \
    launch<AK_, BK_, EPI_F32>(p, s, st);                                                     \
  else                                                                                       \
    launch<AK_, BK_, EPI_STORE>(p, s, st);
  if (a_kc && b_kc) {
    FT_GEMM_LAUNCH(true, true)
  } else if (a_kc && !b_kc) {
    FT_GEMM_LAUNCH(true, false)
  } else if (!a_kc && !b_kc) {
    FT_GEMM_LAUNCH(false, false)
  } else {
    FT_GEMM_LAUNCH(false, true)
  }
#undef FT_GEMM_LAUNCH
  FT_LAUNCH_CHECK();
  if (s > 1) {
    const long MN = M * N;
    hipLaunchKernelGGL(splitk_reduce_kernel, dim3((unsigned)((MN / 8 + 255) / 256)), dim3(256), 0, st,
                       cptr<float>(ws), s, MN, (int)N, mptr<bf16_t>(c), (long)N, rp, (long)N);
    FT_LAUNCH_CHECK();
  }
  return c;
}

// FFN up-projection with the SwiGLU epilogue: x [T, D] @ w13 [2F, D]^T.
// Returns (a = silu(g) * u [T, F], gu = [g | u] [T, 2F]) — gu is what the backward needs.
std::tuple<at::Tensor, at::Tensor> gemm_swiglu(const at::Tensor& x, const at::Tensor& w13) {
  FT_CHECK_CUDA(x);
  FT_CHECK_BF16(x);
  FT_CHECK_BF16(w13);
  FT_CHECK_CONTIG(x);
  FT_CHECK_CONTIG(w13);
  const long D = x.size(-1), T = x.numel() / D, F2 = w13.size(0), F = F2 / 2;
  TORCH_CHECK(w13.size(1) == D, "gemm_swiglu: shape mismatch");
  TORCH_CHECK(T % BM == 0 && F % 128 == 0 && D % BK == 0, "gemm_swiglu: T % 256, F % 128, D % 64 required");
  const at::DeviceGuard guard(x.device());
  auto a = at::empty({T, F}, x.options());
  auto gu = at::empty({T, F2}, x.options());
  GemmArgs p{};
  p.a = cptr<bf16_t>(x);
  p.b = cptr<bf16_t>(w13);
  p.c = mptr<bf16_t>(a);
  p.c2 = mptr<bf16_t>(gu);
  p.lda = D;
  p.ldb = D;
  p.ldc = F;
  p.M = T;
  p.N = F2;
  p.K = D;
  p.tiles_m = T / BM;
  p.tiles_n = F / 128;
  p.k_per_split = D;
  p.ffn = F;
  launch<true, true, EPI_SWIGLU>(p, 1, ft_stream());
  FT_LAUNCH_CHECK();
  return {a, gu};
}

// FFN backward through w2 and SwiGLU: da = dy [T, D] @ w2 [D, F] (B read as [K=D, N=F]),
// then dgu = [dg | du] from the saved gu, in the epilogue. Returns dgu [T, 2F].
at::Tensor gemm_swiglu_bwd(const at::Tensor& dy, const at::Tensor& w2, const at::Tensor& gu) {
  FT_CHECK_CUDA(dy);
  FT_CHECK_BF16(dy);
  FT_CHECK_BF16(w2);
  FT_CHECK_BF16(gu);
  FT_CHECK_CONTIG(dy);
  FT_CHECK_CONTIG(w2);
  FT_CHECK_CONTIG(gu);
  const long D = dy.size(-1), T = dy.numel() / D, F = w2.size(1);
  TORCH_CHECK(w2.size(0) == D && gu.numel() == T * 2 * F, "gemm_swiglu_bwd: shape mismatch");
  TORCH_CHECK(T % BM == 0 && F % BN == 0 && D % BK == 0, "gemm_swiglu_bwd: T, F % 256, D % 64 required");
  const at::DeviceGuard guard(dy.device());
  auto dgu = at::empty({T, 2 * F}, dy.options());
  GemmArgs p{};
  p.a = cptr<bf16_t>(dy);
  p.b = cptr<bf16_t>(w2);
  p.c = mptr<bf16_t>(dgu);
  p.r = cptr<bf16_t>(gu);
  p.lda = D;
  p.ldb = F;
  p.ldc = 2 * F;
  p.ldr = 2 * F;
  p.M = T;
  p.N = F;
  p.K = D;
  p.tiles_m = T / BM;
  p.tiles_n = F / BN;
  p.k_per_split = D;
  p.ffn = F;
  launch<true, false, EPI_SWIGLU_BWD>(p, 1, ft_stream());
  FT_LAUNCH_CHECK();
  return dgu;
}

// Ablation timing hook (scripts/gemm_ablate.py): forward NT layout, no split, ABL as above.
at::Tensor gemm_ablate(const at::Tensor& a, const at::Tensor& b, int64_t M, int64_t N, int64_t K, int64_t abl) {
  TORCH_CHECK(M % BM == 0 && N % BN == 0 && K % BK == 0 && a.numel() == M * K && b.numel() == N * K);
  const at::DeviceGuard guard(a.device());
  auto c = at::empty({M, N}, a.options());
  GemmArgs p{};
  p.a = cptr<bf16_t>(a);
  p.b = cptr<bf16_t>(b);
  p.c = mptr<bf16_t>(c);
  p.lda = K;
  p.ldb = K;
  p.ldc = N;
  p.M = M;
  p.N = N;
  p.K = K;
  p.tiles_m = M / BM;
  p.tiles_n = N / BN;
  p.k_per_split = K;
  const dim3 g(p.tiles_m * p.tiles_n, 1);
  hipStream_t s = ft_stream();
  switch (abl) {
    case 1: hipLaunchKernelGGL((gemm_kernel<true, true, EPI_STORE, false, 1>), g, dim3(NT), 0, s, p); break;
    case 2: hipLaunchKernelGGL((gemm_kernel<true, true, EPI_STORE, false, 2>), g, dim3(NT), 0, s, p); break;
    case 3: hipLaunchKernelGGL((gemm_kernel<true, true, EPI_STORE, false, 3>), g, dim3(NT), 0, s, p); break;
    case 4: hipLaunchKernelGGL((gemm_kernel<true, true, EPI_STORE, false, 4>), g, dim3(NT), 0, s, p); break;
    case 5: hipLaunchKernelGGL((gemm_kernel<true, true, EPI_STORE, false, 5>), g, dim3(NT), 0, s, p); break;
    case 6: hipLaunchKernelGGL((gemm_kernel<true, true, EPI_STORE, false, 6>), g, dim3(NT), 0, s, p); break;
    default: hipLaunchKernelGGL((gemm_kernel<true, true, EPI_STORE, false, 0>), g, dim3(NT), 0, s, p); break;
  }
  FT_LAUNCH_CHECK();
  return c;
}

// A/B hook: tile 0 (per shape) / 128 / 256; asm_reads -1 (unchanged) / 0 / 1.
void gemm_config(int64_t tile, int64_t asm_reads) {
  TORCH_CHECK(tile == 0 || tile == 128 || tile == 256, "gemm_config: tile 0, 128 or 256");
  g_tile = (int)tile;
  if (asm_reads >= 0) g_asm_reads = (int)asm_reads;
}

TORCH_LIBRARY_FRAGMENT(ftamd, m) {
  m.def("gemm_config(int tile, int asm_reads=-1) -> ()", &gemm_config);
  m.def("gemm_ablate(Tensor a, Tensor b, int M, int N, int K, int abl) -> Tensor", &gemm_ablate);
  m.def(
      "gemm(Tensor a, bool a_kc, Tensor b, bool b_kc, int M, int N, int K, Tensor(a!)? out, Tensor? residual, "
      "bool accumulate, int splits) -> Tensor",
      &gemm);
  m.def("gemm_swiglu(Tensor x, Tensor w13) -> (Tensor, Tensor)", &gemm_swiglu);
  m.def("gemm_swiglu_bwd(Tensor dy, Tensor w2, Tensor gu) -> Tensor", &gemm_swiglu_bwd);
}
