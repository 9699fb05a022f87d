// fp32 GEMM on the CDNA4 matrix cores (v_mfma_f32_16x16x4_f32) for --model-dtype fp32: the forward,
// dX and dW products of every nn.Linear (reference model.py:195,215,254,379, utils.py:14-19), which
// the 16-bit w4 / s kernels do not take.
//
//   C[M, N] (+)= sum_k A(m, k) * B(n, k) (+ residual)
//   A(m, k) = a[m * lda + k] (a_t = false) or a[k * lda + m] (a_t = true)
//   B(n, k) = b[n * ldb + k] (b_t = false) or b[k * ldb + n] (b_t = true)
//   forward x W^T: (false, false); dX = dY W: (false, true); dW = dY^T X: (true, true) -- the same
//   layout flags as gemm_w4_ex, so ops/functional.py routes the three products the same way.
//
// Why a different shape from the 16-bit kernels: fp32 MFMA is 1/16 of the bf16 rate per byte of
// operand (16x16x4 = 2 kFLOP per 32-cycle issue from 512 B of operands vs 16x16x32 bf16 = 16 kFLOP
// per 8 cycles from 2 KiB), so the kernel is MFMA-bound with plain LDS traffic and no split-K:
//   * 128 x 128 tile, BK = 32, 4 waves (2 x 2), each a 64 x 64 quadrant = 4 x 4 accumulators of
//     16 x 16; two workgroups per CU (80 KiB of LDS each), so one's barrier / epilogue runs while
//     the other issues MFMAs.
//   * Operands global -> registers (float4, the next K-tile in flight during the current one's
//     MFMAs) -> LDS in the layout they have in HBM: k-contiguous operands as [row][40] (32 k + 8
//     pad: the ds_read_b128 fragment reads are conflict-free), row-contiguous (k-major) ones as
//     [k][132] (lanes 16-31 read 4 k-rows further = 16 banks away). One barrier per K-tile
//     (double-buffered LDS).
//   * K order inside a 16-deep chunk: MFMA j of the chunk takes k = 4 g + j from lane group
//     g = lane / 16, so a lane's four MFMAs read one float4 of its row (k-contiguous images).
//   * Grids of less than one tile per CU (the GPT-2-sized products: 96 tiles at T = 2048) split K
//     into S slices: each writes its raw fp32 partial to a workspace and a reduction pass sums the
//     slices in order 0 .. S-1 (deterministic) and applies the epilogue.
//   * Epilogue from the accumulators: 16 lanes store 64 contiguous bytes of a row; optional
//     accumulate (gradient accumulation), + residual (fused residual add), and one sum-of-squares
//     partial per tile for the global gradient norm (as the w4 dW epilogue: part[tn * tiles_m + tm]).
//   * Tiles XCD-contiguous (workgroup t on XCD t % 8 takes a contiguous M-fastest range), so an
//     operand panel is shared through one L2.
#include "torch_utils.h"

namespace {

constexpr int BM = 128, BN = 128, BK = 32, NT = 256;
constexpr int SK = BK + 8;    // floats per row of a k-contiguous image
constexpr int SR = BM + 4;    // floats per k-row of a row-contiguous image
constexpr int IMG = BM * SK;  // floats per operand image (5120 >= BK * SR = 4224)
static_assert(BK * SR <= IMG, "image size");
constexpr int LDS_FLOATS = 2 * 2 * IMG;  // 2 stages x (A, B): 80 KiB

struct F32Args {
  const float* a;
  const float* b;
  float* c;
  const float* r;  // residual [M, N] or null
  float* part;     // per-tile sums of squares or null
  long lda, ldb, ldc, ldr;
  int M, N, K;
  int tiles_m, tiles_n, part_n;
  int acc;  // C += instead of C =
  int ks;     // K slices (1: none)
  float* ws;  // ks > 1: raw partials [ks][M][N]
};

__device__ __forceinline__ void tile_of(int t, int tiles_m, int tiles_n, int& tm, int& tn) {
  const int nwg = tiles_m * tiles_n;
  const int q = nwg / 8, rem = nwg % 8;
  const int x = t % 8, o = t / 8;
  const int w = (x < rem ? x * (q + 1) : rem * (q + 1) + (x - rem) * q) + o;
  tm = w % tiles_m;
  tn = w / tiles_m;
}

// One operand's K-tile: global -> 4 float4 registers per thread. RC (row-contiguous, k-major):
// 32 k-rows x 32 float4; otherwise 128 rows x 8 float4. Rows past `rows` are clamped (their
// products land in C rows / columns that are never stored) or, row-contiguous, zero-filled
// (rows % 4 == 0, checked on the host, keeps a float4 inside or outside).
template <bool RC>
__device__ __forceinline__ void load_tile(const float* __restrict__ x, long ld, int i0, int rows, int k0, int tid,
                                          float4 (&v)[4]) {
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int idx = q * NT + tid;
    if constexpr (RC) {
      const int k = idx >> 5, c4 = idx & 31;
      const int i = i0 + 4 * c4;
      v[q] = i < rows ? *reinterpret_cast<const float4*>(x + (long)(k0 + k) * ld + i) : make_float4(0.f, 0.f, 0.f, 0.f);
    } else {
      const int row = idx >> 3, c4 = idx & 7;
      const int i = min(i0 + row, rows - 1);
      v[q] = *reinterpret_cast<const float4*>(x + (long)i * ld + k0 + 4 * c4);
    }
  }
}

template <bool RC>
__device__ __forceinline__ void store_tile(float* img, int tid, const float4 (&v)[4]) {
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int idx = q * NT + tid;
    if constexpr (RC)
      *reinterpret_cast<float4*>(img + (idx >> 5) * SR + 4 * (idx & 31)) = v[q];
    else
      *reinterpret_cast<float4*>(img + (idx >> 3) * SK + 4 * (idx & 7)) = v[q];
  }
}

// f[j] = X(row base + lane % 16, k = 16 c + 4 (lane / 16) + j) from an image
template <bool RC>
__device__ __forceinline__ float4 frag(const float* img, int base, int c, int lane) {
  const int r16 = lane & 15, g = lane >> 4;
  if constexpr (RC) {
    const float* p = img + (16 * c + 4 * g) * SR + base + r16;
    return make_float4(p[0], p[SR], p[2 * SR], p[3 * SR]);
  } else {
    return *reinterpret_cast<const float4*>(img + (base + r16) * SK + 16 * c + 4 * g);
  }
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// The epilogue of a K slice's 128 x 128 tile: raw partial (split-K) or C (+)= acc (+ residual), with
// the tile's sum-of-squares partial through `red` (>= 4 floats of LDS no wave still reads).
template <bool RES, bool PART>
__device__ __forceinline__ void epilogue(const F32Args& p, f32x4_t (&acc)[4][4], int slice, int tm, int tn,
                                         int wm, int wn, int lane, int wid, int tid, float* red) {
  const int m0 = tm * BM, n0 = tn * BN;
  // epilogue: acc[i][j][v] = C(m0 + 64 wm + 16 i + 4 (lane / 16) + v, n0 + 64 wn + 16 j + lane % 16)
  const int g = lane >> 4, r16 = lane & 15;
  if (p.ks > 1) {  // a slice's raw partial (f32_splitk_reduce applies the epilogue)
    float* w = p.ws + (long)slice * p.M * p.N;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const int m = m0 + wm * 64 + i * 16 + 4 * g + v;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int n = n0 + wn * 64 + j * 16 + r16;
          if (m < p.M && n < p.N) w[(long)m * p.N + n] = acc[i][j][v];
        }
      }
    return;
  }
  float sq = 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const int m = m0 + wm * 64 + i * 16 + 4 * g + v;
      if (m >= p.M) continue;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int n = n0 + wn * 64 + j * 16 + r16;
        if (n >= p.N) continue;
        float* cp = p.c + (long)m * p.ldc + n;
        float x = acc[i][j][v];
        if (p.acc) x += *cp;
        if constexpr (RES) x += p.r[(long)m * p.ldr + n];
        if constexpr (PART) sq = fmaf(x, x, sq);
        *cp = x;
      }
    }
  if constexpr (PART) {  // one partial per tile, fixed order (deterministic)
    sq = wave_sum(sq);
    if (lane == 0) red[wid] = sq;
    __syncthreads();
    if (tid == 0) p.part[tn * p.tiles_m + tm] = (red[0] + red[1]) + (red[2] + red[3]);
    // slots past this grid (the sink's buffer is sized for any producer): zero, or stale partials
    // of an earlier producer would enter the norm
    if (blockIdx.x == 0)
      for (int s = p.tiles_m * p.tiles_n + tid; s < p.part_n; s += NT) p.part[s] = 0.f;
  }
}

template <bool AT, bool BT, bool RES, bool PART>
__global__ __launch_bounds__(NT, 2) void gemm_f32_kernel(F32Args p) {
  __shared__ __attribute__((aligned(16))) float smem[LDS_FLOATS];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid >> 1, wn = wid & 1;
  const int ntile = p.tiles_m * p.tiles_n;
  const int slice = blockIdx.x / ntile;
  int tm, tn;
  tile_of(blockIdx.x - slice * ntile, p.tiles_m, p.tiles_n, tm, tn);
  const int m0 = tm * BM, n0 = tn * BN;
  const int nk_all = p.K / BK, per = (nk_all + p.ks - 1) / p.ks;
  const int kb = slice * per * BK;  // this slice's first k
  const int nk = min(per, nk_all - slice * per);

  f32x4_t acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  float4 ra[4], rb[4];
  load_tile<AT>(p.a, p.lda, m0, p.M, kb, tid, ra);
  load_tile<BT>(p.b, p.ldb, n0, p.N, kb, tid, rb);
  store_tile<AT>(smem, tid, ra);
  store_tile<BT>(smem + IMG, tid, rb);
  __syncthreads();

  // fragment registers of the two 16-deep chunks of a K-tile: chunk 1 is read before the barrier
  // and multiplied after it, under the next K-tile's chunk-0 reads (the LDS latency and the
  // barrier's skew hide under 64 MFMAs instead of stalling every wave at the top of the tile)
  float4 fa[2][4], fb[2][4];
  auto read = [&](const float* ia, int c, float4 (&xa)[4], float4 (&xb)[4]) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < 4; ++i) xa[i] = frag<AT>(ia, wm * 64 + i * 16, c, lane);
#pragma unroll
    for (int j = 0; j < 4; ++j) xb[j] = frag<BT>(ia + IMG, wn * 64 + j * 16, c, lane);
  };
  auto mma = [&](const float4 (&xa)[4], const float4 (&xb)[4]) __attribute__((always_inline)) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float av = q == 0 ? xa[i].x : q == 1 ? xa[i].y : q == 2 ? xa[i].z : xa[i].w;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float bv = q == 0 ? xb[j].x : q == 1 ? xb[j].y : q == 2 ? xb[j].z : xb[j].w;
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, acc[i][j], 0, 0, 0);
        }
      }
    }
  };
  static_assert(BK == 32, "two 16-deep chunks per K-tile");
  read(smem, 0, fa[0], fb[0]);
  for (int kt = 0; kt < nk; ++kt) {
    const float* cur = smem + (kt & 1) * 2 * IMG;
    float* nxt = smem + ((kt + 1) & 1) * 2 * IMG;
    // the next K-tile's loads in flight under this one's MFMAs; unconditional (the last iteration
    // reloads its own tile into the idle buffer): with the loads and stores under a branch the
    // compiler parked the prefetch registers in scratch memory, waiting on each load at once
    const int kn = kb + min(kt + 1, nk - 1) * BK;
    load_tile<AT>(p.a, p.lda, m0, p.M, kn, tid, ra);
    load_tile<BT>(p.b, p.ldb, n0, p.N, kn, tid, rb);
    read(cur, 1, fa[1], fb[1]);
    mma(fa[0], fb[0]);
    store_tile<AT>(nxt, tid, ra);
    store_tile<BT>(nxt + IMG, tid, rb);
    __syncthreads();
    read(nxt, 0, fa[0], fb[0]);  // (after the last K-tile: a harmless read of the idle buffer)
    mma(fa[1], fb[1]);
  }
  __syncthreads();  // every wave's last (idle-buffer) reads are done before smem is reused

  epilogue<RES, PART>(p, acc, slice, tm, tn, wm, wn, lane, wid, tid, smem);
}

// ---- LDS-DMA form (default): the operands go HBM -> LDS by buffer_load_dwordx4 ... lds, never
// through VGPRs (a register round trip's returning loads compete with the MFMAs for the register
// file). 16 KiB images without padding, the bank spread done by the DMA's per-lane source address:
//   k-contiguous [row][32]: 128-B rows, row r's 16-B slot s holds chunk s ^ (r & 7) (ds_read_b128
//     fragment reads conflict-free);
//   k-major [k][128]: 512-B k-rows, k-row k's slot s holds chunk s ^ 4 [k & 4] (lanes 16-31, 4
//     k-rows further, 16 banks away for ds_read_b32).
// A wave's DMA instruction fills 1 KiB (piece P = 8 rows / 2 k-rows); 4 + 4 per wave per K-tile.
// Tails are clamped onto the last valid row (their products only reach C entries never stored);
// every byte offset stays below 4 GiB (host check; 32-bit buffer offsets).
constexpr int DIMG = 4096;  // floats per operand image (16 KiB)
typedef int i32x4_t __attribute__((ext_vector_type(4)));

__device__ __forceinline__ unsigned lds_u32(const void* q) {
  return (unsigned)(uintptr_t)((const __attribute__((address_space(3))) char*)q);
}

__device__ __forceinline__ i32x4_t make_srd(const void* q) {
  const unsigned long long a = (unsigned long long)q;
  i32x4_t r;
  r[0] = __builtin_amdgcn_readfirstlane((int)(unsigned)a);
  r[1] = __builtin_amdgcn_readfirstlane((int)((unsigned)(a >> 32) & 0xffffu));
  r[2] = -1;
  r[3] = 0x00020000;
  return r;
}

// 16 B per lane from srd + voff + soff into LDS [sbase + 16 * lane] (m0 = sbase; nothing else in
// the kernel uses m0; s_mov does not touch SCC)
__device__ __forceinline__ void dma16(const i32x4_t& srd, unsigned voff, unsigned soff, unsigned sbase) {
  asm volatile("s_mov_b32 m0, %2\n\tbuffer_load_dwordx4 %0, %1, %3 offen lds"
               :
               : "v"(voff), "s"(srd), "s"(sbase), "s"(soff)
               : "memory");
}

// per-lane source offsets (bytes, without the K-tile's soff) of the 4 pieces a wave fills
template <bool RC>
__device__ __forceinline__ void dma_offsets(long ld, int i0, int rows, int wid, int lane, unsigned (&vo)[4]) {
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int P = q * 4 + wid;
    if constexpr (RC) {
      const int k = 2 * P + (lane >> 5);
      const int c = (lane & 31) ^ (((k >> 2) & 1) * 4);
      const int i = min(i0 + 4 * c, rows - 4);
      vo[q] = (unsigned)(((long)k * ld + i) * 4);
    } else {
      const int r = 8 * P + (lane >> 3);
      const int c = (lane & 7) ^ (r & 7);
      const int i = min(i0 + r, rows - 1);
      vo[q] = (unsigned)(((long)i * ld + 4 * c) * 4);
    }
  }
}

// f[j] = X(row base + lane % 16, k = 16 c + 4 (lane / 16) + j) from a swizzled image
template <bool RC>
__device__ __forceinline__ float4 dfrag(const float* img, int base, int c, int lane) {
  const int r16 = lane & 15, g = lane >> 4;
  if constexpr (RC) {
    const int m = base + r16;
    const float* q = img + (16 * c + 4 * g) * 128 + ((((m >> 2) ^ ((g & 1) * 4))) << 2) + (m & 3);
    return make_float4(q[0], q[128], q[256], q[384]);  // (k + 1 .. k + 3 share bit 2 of k: same swizzle)
  } else {
    const int r = base + r16;
    return *reinterpret_cast<const float4*>(img + r * 32 + (((4 * c + g) ^ (r & 7)) << 2));
  }
}

template <bool AT, bool BT, bool RES, bool PART>
__global__ __launch_bounds__(NT, 2) void gemm_f32d_kernel(F32Args p) {
  __shared__ __attribute__((aligned(1024))) float smem[2 * 2 * DIMG];  // 2 stages x (A, B): 64 KiB
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid >> 1, wn = wid & 1;
  const int ntile = p.tiles_m * p.tiles_n;
  const int slice = blockIdx.x / ntile;
  int tm, tn;
  tile_of(blockIdx.x - slice * ntile, p.tiles_m, p.tiles_n, tm, tn);
  const int m0 = tm * BM, n0 = tn * BN;
  const int nk_all = p.K / BK, per = (nk_all + p.ks - 1) / p.ks;
  const int kb = slice * per * BK;
  const int nk = min(per, nk_all - slice * per);

  const i32x4_t srdA = make_srd(p.a), srdB = make_srd(p.b);
  unsigned voA[4], voB[4];
  dma_offsets<AT>(p.lda, m0, p.M, wid, lane, voA);
  dma_offsets<BT>(p.ldb, n0, p.N, wid, lane, voB);
  // soff of K-tile t: k-major operands advance by BK rows, k-contiguous ones by BK columns
  const unsigned stA = AT ? (unsigned)(BK * p.lda * 4) : (unsigned)(BK * 4);
  const unsigned stB = BT ? (unsigned)(BK * p.ldb * 4) : (unsigned)(BK * 4);
  const unsigned sA0 = AT ? (unsigned)((long)kb * p.lda * 4) : (unsigned)(kb * 4);
  const unsigned sB0 = BT ? (unsigned)((long)kb * p.ldb * 4) : (unsigned)(kb * 4);
  const unsigned lds0 = __builtin_amdgcn_readfirstlane(lds_u32(smem));
  auto issue = [&](int t, int stage) __attribute__((always_inline)) {
    const unsigned ba = lds0 + (unsigned)(stage * 2 * DIMG * 4), bb = ba + DIMG * 4;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const unsigned piece = (unsigned)((q * 4 + wid) * 1024);
      dma16(srdA, voA[q], sA0 + t * stA, __builtin_amdgcn_readfirstlane(ba + piece));
      dma16(srdB, voB[q], sB0 + t * stB, __builtin_amdgcn_readfirstlane(bb + piece));
    }
  };

  f32x4_t acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  issue(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const float* cur = smem + (kt & 1) * 2 * DIMG;
    if (kt + 1 < nk) issue(kt + 1, (kt + 1) & 1);  // (uniform) into the stage read last iteration
#pragma unroll
    for (int c = 0; c < BK / 16; ++c) {
      float4 fa[4], fb[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) fa[i] = dfrag<AT>(cur, wm * 64 + i * 16, c, lane);
#pragma unroll
      for (int j = 0; j < 4; ++j) fb[j] = dfrag<BT>(cur + DIMG, wn * 64 + j * 16, c, lane);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float av = q == 0 ? fa[i].x : q == 1 ? fa[i].y : q == 2 ? fa[i].z : fa[i].w;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const float bv = q == 0 ? fb[j].x : q == 1 ? fb[j].y : q == 2 ? fb[j].z : fb[j].w;
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, acc[i][j], 0, 0, 0);
          }
        }
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the next K-tile's DMA landed (this wave's) ...
    __syncthreads();                                   // ... and everyone's; cur is free again
  }
  epilogue<RES, PART>(p, acc, slice, tm, tn, wm, wn, lane, wid, tid, smem);
}

// Sums the ks slice partials of one 128 x 128 tile in slice order and applies the epilogue
// (accumulate, residual, the tile's sum-of-squares partial), as gemm_f32_kernel's. 1024 threads
// per tile (the split grids have few tiles: 96 at the GPT-2 sizes), float4 when the rows allow.
constexpr int RT = 1024;

template <bool RES, bool PART>
__global__ __launch_bounds__(RT) void f32_splitk_reduce(F32Args p) {
  __shared__ float red[RT / 64];
  // without the tile's sum-of-squares partial a tile is 4 workgroups of 32 rows (the grids that split
  // have few tiles: 4x the memory parallelism); with it, one workgroup sums the whole tile
  constexpr int RS = PART ? 1 : 4, RB = BM / RS;
  const int tid = threadIdx.x;
  const int tile = blockIdx.x / RS, rb = (blockIdx.x % RS) * RB;
  const int tm = tile % p.tiles_m, tn = tile / p.tiles_m;
  const long mn = (long)p.M * p.N;
  const bool vec = (p.N % 4 == 0) && (p.ldc % 4 == 0) && (!RES || p.ldr % 4 == 0);  // uniform
  float sq = 0.f;
  if (vec) {
#pragma unroll
    for (int q = 0; q < RB * BN / 4 / RT; ++q) {
      const int e = q * RT + tid;
      const int m = tm * BM + rb + e / (BN / 4), n = tn * BN + 4 * (e % (BN / 4));
      if (m >= p.M || n >= p.N) continue;
      const float* w = p.ws + (long)m * p.N + n;
      float4 x = *reinterpret_cast<const float4*>(w);
      for (int s = 1; s < p.ks; ++s) {
        const float4 y = *reinterpret_cast<const float4*>(w + s * mn);
        x.x += y.x; x.y += y.y; x.z += y.z; x.w += y.w;
      }
      float4* cp = reinterpret_cast<float4*>(p.c + (long)m * p.ldc + n);
      if (p.acc) {
        const float4 c0 = *cp;
        x.x += c0.x; x.y += c0.y; x.z += c0.z; x.w += c0.w;
      }
      if constexpr (RES) {
        const float4 r = *reinterpret_cast<const float4*>(p.r + (long)m * p.ldr + n);
        x.x += r.x; x.y += r.y; x.z += r.z; x.w += r.w;
      }
      if constexpr (PART) sq = fmaf(x.w, x.w, fmaf(x.z, x.z, fmaf(x.y, x.y, fmaf(x.x, x.x, sq))));
      *cp = x;
    }
  } else {
    for (int e = tid; e < RB * BN; e += RT) {
      const int m = tm * BM + rb + e / BN, n = tn * BN + e % BN;
      if (m >= p.M || n >= p.N) continue;
      const float* w = p.ws + (long)m * p.N + n;
      float x = w[0];
      for (int s = 1; s < p.ks; ++s) x += w[s * mn];
      float* cp = p.c + (long)m * p.ldc + n;
      if (p.acc) x += *cp;
      if constexpr (RES) x += p.r[(long)m * p.ldr + n];
      if constexpr (PART) sq = fmaf(x, x, sq);
      *cp = x;
    }
  }
  if constexpr (PART) {
    sq = wave_sum(sq);
    if ((tid & 63) == 0) red[tid >> 6] = sq;
    __syncthreads();
    if (tid == 0) {
      float t = 0.f;
      for (int w = 0; w < RT / 64; ++w) t += red[w];  // fixed order
      p.part[tn * p.tiles_m + tm] = t;
    }
    if (blockIdx.x == 0)
      for (int s = p.tiles_m * p.tiles_n + tid; s < p.part_n; s += RT) p.part[s] = 0.f;
  }
}

// K slices: -1 automatic, 0 / 1 none, > 1 forced where K allows (gemm_f32_set_splitk, for A/B)
int g_f32_splitk = -1;

// (every slice non-empty: ceil(nk / ceil(nk / s)) slices of ceil(nk / s) K-tiles, the last shorter)
int f32_slices(int ntile, int nk_all) {
  int s = 1;
  if (g_f32_splitk >= 0) {
    s = std::max(1, std::min(g_f32_splitk, nk_all));
  } else if (ntile < 256) {  // less than a tile per CU: enough workgroups for two per CU, slices of
    for (int c : {2, 3, 4, 6, 8})  // at least 8 K-tiles (256 deep)
      if ((long)ntile * c <= 512 && nk_all / c >= 8) s = c;
  }
  const int per = (nk_all + s - 1) / s;
  return (nk_all + per - 1) / per;
}

// LDS-DMA form (default) or the register round-trip form (gemm_f32_set_dma, A/B; also taken when an
// operand exceeds 32-bit buffer offsets)
int g_f32_dma = 1;

template <bool AT, bool BT>
void launch_lay(const F32Args& p, bool res, bool part, bool dma, hipStream_t st) {
  const dim3 g(p.tiles_m * p.tiles_n * p.ks), b(NT);
  if (dma) {
    if (p.ks > 1 || (!res && !part))
      hipLaunchKernelGGL((gemm_f32d_kernel<AT, BT, false, false>), g, b, 0, st, p);
    else if (res && part)
      hipLaunchKernelGGL((gemm_f32d_kernel<AT, BT, true, true>), g, b, 0, st, p);
    else if (res)
      hipLaunchKernelGGL((gemm_f32d_kernel<AT, BT, true, false>), g, b, 0, st, p);
    else
      hipLaunchKernelGGL((gemm_f32d_kernel<AT, BT, false, true>), g, b, 0, st, p);
  }
  if (p.ks > 1) {  // slices write raw partials: one instantiation, then the reduction's epilogue
    if (!dma) hipLaunchKernelGGL((gemm_f32_kernel<AT, BT, false, false>), g, b, 0, st, p);
    const dim3 gr(p.tiles_m * p.tiles_n * (part ? 1 : 4)), br(RT);  // (RS of f32_splitk_reduce)
    if (res && part)
      hipLaunchKernelGGL((f32_splitk_reduce<true, true>), gr, br, 0, st, p);
    else if (res)
      hipLaunchKernelGGL((f32_splitk_reduce<true, false>), gr, br, 0, st, p);
    else if (part)
      hipLaunchKernelGGL((f32_splitk_reduce<false, true>), gr, br, 0, st, p);
    else
      hipLaunchKernelGGL((f32_splitk_reduce<false, false>), gr, br, 0, st, p);
    return;
  }
  if (dma) return;
  if (res && part)
    hipLaunchKernelGGL((gemm_f32_kernel<AT, BT, true, true>), g, b, 0, st, p);
  else if (res)
    hipLaunchKernelGGL((gemm_f32_kernel<AT, BT, true, false>), g, b, 0, st, p);
  else if (part)
    hipLaunchKernelGGL((gemm_f32_kernel<AT, BT, false, true>), g, b, 0, st, p);
  else
    hipLaunchKernelGGL((gemm_f32_kernel<AT, BT, false, false>), g, b, 0, st, p);
}

long ld_of(const at::Tensor& t, const char* name) {
  TORCH_CHECK(t.dim() == 2 && t.stride(1) == 1, "gemm_f32: ", name, " must be 2-D with unit column stride");
  TORCH_CHECK(t.stride(0) % 4 == 0 && reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0,
              "gemm_f32: ", name, " rows must be 16-byte aligned");
  return t.stride(0);
}

}  // namespace

// C[M, N] (+)= A B^T over K (layouts above), fp32. K % 32 == 0; a k-major (transposed) operand needs
// its row count % 4 == 0. out: written (or accumulated) in place and returned; part: per-tile
// sums of squares of the stored C (>= ceil(M / 128) * ceil(N / 128) slots); residual: [M, N] added.
at::Tensor gemm_f32(const at::Tensor& a, bool a_t, const at::Tensor& b, bool b_t, int64_t M, int64_t N, int64_t K,
                    const std::optional<at::Tensor>& out, bool accumulate, const std::optional<at::Tensor>& part,
                    const std::optional<at::Tensor>& residual) {
  FT_CHECK_CUDA(a);
  FT_CHECK_F32(a);
  FT_CHECK_F32(b);
  TORCH_CHECK(M > 0 && N > 0 && K > 0 && K % BK == 0, "gemm_f32: K must be a positive multiple of 32");
  TORCH_CHECK(a.size(0) == (a_t ? K : M) && a.size(1) == (a_t ? M : K), "gemm_f32: a shape");
  TORCH_CHECK(b.size(0) == (b_t ? K : N) && b.size(1) == (b_t ? N : K), "gemm_f32: b shape");
  TORCH_CHECK(!a_t || M % 4 == 0, "gemm_f32: a k-major A needs M % 4 == 0");
  TORCH_CHECK(!b_t || N % 4 == 0, "gemm_f32: a k-major B needs N % 4 == 0");
  const at::DeviceGuard guard(a.device());
  F32Args p{};
  p.a = cptr<float>(a);
  p.b = cptr<float>(b);
  p.lda = ld_of(a, "a");
  p.ldb = ld_of(b, "b");
  at::Tensor c;
  if (out.has_value() && out->defined()) {
    c = *out;
    FT_CHECK_F32(c);
    TORCH_CHECK(c.size(0) == M && c.size(1) == N, "gemm_f32: out shape");
    p.ldc = ld_of(c, "out");
  } else {
    TORCH_CHECK(!accumulate, "gemm_f32: accumulate needs out");
    c = at::empty({M, N}, a.options());
    p.ldc = N;
  }
  p.c = mptr<float>(c);
  p.acc = accumulate ? 1 : 0;
  p.M = (int)M;
  p.N = (int)N;
  p.K = (int)K;
  p.tiles_m = (int)((M + BM - 1) / BM);
  p.tiles_n = (int)((N + BN - 1) / BN);
  const bool res = residual.has_value() && residual->defined();
  if (res) {
    FT_CHECK_F32((*residual));
    TORCH_CHECK(residual->size(0) == M && residual->size(1) == N, "gemm_f32: residual shape");
    p.r = cptr<float>(*residual);
    p.ldr = ld_of(*residual, "residual");
  }
  const bool pt = part.has_value() && part->defined();
  if (pt) {
    FT_CHECK_F32((*part));
    FT_CHECK_CONTIG((*part));
    TORCH_CHECK(part->numel() >= (long)p.tiles_m * p.tiles_n, "gemm_f32: part holds ", part->numel(),
                " partials, need ", (long)p.tiles_m * p.tiles_n);
    p.part = mptr<float>(*part);
    p.part_n = (int)part->numel();
  }
  p.ks = f32_slices(p.tiles_m * p.tiles_n, p.K / BK);
  at::Tensor ws;
  if (p.ks > 1) {
    ws = at::empty({(long)p.ks, M, N}, a.options());
    p.ws = mptr<float>(ws);
  }
  // the DMA form's 32-bit buffer offsets: every operand byte within 4 GiB of its base
  const auto fits = [](const at::Tensor& t) { return (double)t.stride(0) * t.size(0) * 4.0 < 4294967296.0; };
  const bool dma = g_f32_dma && fits(a) && fits(b);
  const hipStream_t st = ft_stream();
  if (a_t) {
    if (b_t) launch_lay<true, true>(p, res, pt, dma, st); else launch_lay<true, false>(p, res, pt, dma, st);
  } else {
    if (b_t) launch_lay<false, true>(p, res, pt, dma, st); else launch_lay<false, false>(p, res, pt, dma, st);
  }
  FT_LAUNCH_CHECK();
  return c;
}

void gemm_f32_set_splitk(int64_t s) { g_f32_splitk = (int)s; }
void gemm_f32_set_dma(int64_t on) { g_f32_dma = (int)on; }
int64_t gemm_f32_slices(int64_t M, int64_t N, int64_t K) {
  return f32_slices((int)(((M + BM - 1) / BM) * ((N + BN - 1) / BN)), (int)(K / BK));
}

TORCH_LIBRARY_FRAGMENT(ftamd, m) {
  m.def("gemm_f32_set_splitk(int s) -> ()", &gemm_f32_set_splitk);
  m.def("gemm_f32_set_dma(int on) -> ()", &gemm_f32_set_dma);
  m.def("gemm_f32_slices(int M, int N, int K) -> int", &gemm_f32_slices);
  m.def(
      "gemm_f32(Tensor a, bool a_t, Tensor b, bool b_t, int M, int N, int K, Tensor(a!)? out=None, "
      "bool accumulate=False, Tensor(b!)? part=None, Tensor? residual=None) -> Tensor",
      &gemm_f32);
}
