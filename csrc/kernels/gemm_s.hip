// 128 x 128-tile bf16 / fp16 GEMM for gfx950, two workgroups per CU (the "s" kernel): the GPT-2-sized
// projections (M = 2048 tokens, N and K = 768 ... 4096) that the 256-wide tiles underfill.
//
//   C[M, N] = sum_k A(m, k) * B(n, k) (+ residual)   A = [M, K], B = [N, K] row-major (K contiguous)
//   (x W^T of every nn.Linear: reference model.py:195,215,254)
//
// A GPT-2-small projection is 2-13 GFLOP: at the chip's ~2.1 PF/s MFMA ceiling that is 1-6 us, so
// the time goes to filling the chip and to per-tile fixed costs. Structure:
//   * 128 x 128 tile, BK = 64, 4 waves (2 x 2), each a 64 x 64 quadrant = 4 x 4 fragments of
//     v_mfma_f32_16x16x32_bf16 (_f16), accumulators pinned in AGPRs ("+a" asm operands, as gemm_w4).
//     2048 x 768 outputs are 96 tiles, 2048 x 2304 are 288: with two resident workgroups per CU
//     (64 KiB of LDS, <= 128 VGPR + 64 AGPR each) a launch is at most ~1.1 rounds, and one
//     workgroup's barrier / DMA waits and epilogue run while the other issues MFMAs.
//   * A and B by LDS-DMA (global_load_lds_dwordx4: 1 KiB = 8 rows x 128 B per wave-instruction,
//     per-lane source chunk XOR-swizzled by row so the ds_read_b128 fragment reads are
//     conflict-free), double-buffered, tile t+1 in flight while tile t is read; fragment reads by
//     inline asm with explicit lgkmcnt waits (a compiler-placed wait would also drain the DMA).
//   * Optional split-K (ks > 1, explicit only): slice s of K writes fp32 partials; the last-arriving
//     workgroup of a tile (atomic ticket) sums the slices in fixed order 0..ks-1 (deterministic) and
//     applies the epilogue.
//   * Epilogue through LDS (the stage buffers are free after the last K-tile): rows of 256 B,
//     16-B chunks XOR-swizzled by row; whole-row 16-B stores; optional + residual.
//   * Tiles mapped M-fastest inside an XCD's contiguous range (blockIdx % 8 = XCD), so a B panel
//     is shared through one L2.
#include "torch_utils.h"

#include <utility>

namespace {

typedef int i32x4_t __attribute__((ext_vector_type(4)));

template <typename F, int... I>
__device__ __forceinline__ void sfor_impl(F&& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, typename F>
__device__ __forceinline__ void sfor(F&& f) {
  sfor_impl(f, std::make_integer_sequence<int, N>{});
}

constexpr int BM = 128, BN = 128, BK = 64, NT = 256;
constexpr int PIECE = 1024;           // one LDS-DMA wave-instruction: 8 image rows of 128 B
constexpr int OPI = 16 * PIECE;       // one operand image: 128 rows x 128 B
constexpr int STAGE = 2 * OPI;        // A | B
constexpr int LDS_BYTES = 2 * STAGE;  // two stages = 64 KiB

__device__ __forceinline__ unsigned lds_u32(const void* p) {
  return (unsigned)(uintptr_t)((const __attribute__((address_space(3))) char*)p);
}

__device__ __forceinline__ i32x4_t make_srd(const void* p) {
  const unsigned long long a = (unsigned long long)p;
  i32x4_t r;
  r[0] = __builtin_amdgcn_readfirstlane((int)(unsigned)a);
  r[1] = __builtin_amdgcn_readfirstlane((int)((unsigned)(a >> 32) & 0xffffu));
  r[2] = -1;
  r[3] = 0x00020000;
  return r;
}

// LDS-DMA: 16 B per lane from srd + voff + soff into LDS [m0 + 16 * lane], m0 = sbase + IMM
template <int IMM>
__device__ __forceinline__ void dma16(const i32x4_t& srd, unsigned voff, unsigned soff, unsigned sbase) {
  asm volatile("s_add_u32 m0, %2, %4\n\tbuffer_load_dwordx4 %0, %1, %3 offen lds"
               :
               : "v"(voff), "s"(srd), "s"(sbase), "s"(soff), "i"(IMM)
               : "memory", "scc");
}

template <int OFF>
__device__ __forceinline__ void ds16(bf16x8_t& d, unsigned addr) {
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(d) : "v"(addr), "i"(OFF) : "memory");
}

template <class E>
__device__ __forceinline__ void mfma(f32x4_t& c, const bf16x8_t& a, const bf16x8_t& b) {
  if constexpr (std::is_same<E, EF16>::value)
    asm volatile("v_mfma_f32_16x16x32_f16 %0, %1, %2, %0" : "+a"(c) : "v"(a), "v"(b));
  else
    asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(c) : "v"(a), "v"(b));
}

template <int N>
__device__ __forceinline__ void lgkm() {
  asm volatile("s_waitcnt lgkmcnt(%0)" ::"i"(N) : "memory");
}
template <int N>
__device__ __forceinline__ void vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"i"(N) : "memory");
}
__device__ __forceinline__ void barrier() { asm volatile("s_barrier" ::: "memory"); }
__device__ __forceinline__ void tie(bf16x8_t& x) { asm volatile("" : "+v"(x)); }

struct SArgs {
  const bf16_t* a;
  const bf16_t* b;
  bf16_t* c;
  const bf16_t* r;      // residual (may alias c) or null
  float* ws;            // split-K: fp32 partials [KS][tiles][BM * BN]
  unsigned* tickets;    // split-K: per-tile arrival counters (zero; reset by the last arrival)
  long lda, ldb, ldc, ldr;
  int M, N, K;
  int tiles_m, tiles_n, ks;  // split-K factor (1 = none)
};

__device__ __forceinline__ void tile_of(int t, int tiles_m, int tiles_n, int& tm, int& tn) {
  const int nwg = tiles_m * tiles_n;
  const int q = nwg / 8, rem = nwg % 8;
  const int x = t % 8, o = t / 8;
  const int w = (x < rem ? x * (q + 1) : rem * (q + 1) + (x - rem) * q) + o;
  tm = w % tiles_m;
  tn = w / tiles_m;
}

template <class E, bool RES>
__global__ __launch_bounds__(NT, 2) void gemm_s_kernel(SArgs p) {
  __shared__ __attribute__((aligned(1024))) char smem[LDS_BYTES];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid >> 1, wn = wid & 1;
  const int ntile = p.tiles_m * p.tiles_n;
  const int tile = blockIdx.x % ntile, slice = blockIdx.x / ntile;
  int tm, tn;
  tile_of(tile, p.tiles_m, p.tiles_n, tm, tn);
  const int m0 = tm * BM, n0 = tn * BN;
  const int nk_all = p.K / BK;
  const int per = (nk_all + p.ks - 1) / p.ks;
  const int kt0 = slice * per, nk = min(per, nk_all - kt0);

  // LDS-DMA sources: instruction q of wave w covers image rows (q * 4 + w) * 8 + (lane >> 3);
  // lane's 16-B chunk (lane & 7) holds global chunk (lane & 7) ^ (row & 7)
  const i32x4_t srdA = make_srd(p.a + (long)m0 * p.lda + (long)kt0 * BK);
  const i32x4_t srdB = make_srd(p.b + (long)n0 * p.ldb + (long)kt0 * BK);
  const int lrow = wid * 8 + (lane >> 3), lch = (lane & 7) ^ (lane >> 3);
  unsigned voA[4], voB[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    voA[q] = (unsigned)(((q * 32 + lrow) * p.lda + lch * 8) * 2);
    voB[q] = (unsigned)(((q * 32 + lrow) * p.ldb + lch * 8) * 2);
  }
  const unsigned lds0 = __builtin_amdgcn_readfirstlane(lds_u32(smem));
  // fragment reads: lane reads row r0 + (lane & 15), chunk (kk * 4 + (lane >> 4)) ^ (lane & 7)
  const unsigned lrowb = (unsigned)(((lane & 15) >> 3) * PIECE + (lane & 7) * 128);
  const unsigned rdA = lds0 + wm * 8 * PIECE + lrowb;
  const unsigned rdB = lds0 + OPI + wn * 8 * PIECE + lrowb;
  const unsigned ch0 = (unsigned)((((lane >> 4)) ^ (lane & 7)) << 4);
  const unsigned ch1 = (unsigned)(((4 + (lane >> 4)) ^ (lane & 7)) << 4);

  auto issue = [&](int t, unsigned stage) {
    const unsigned sb = __builtin_amdgcn_readfirstlane(lds0 + stage * STAGE + wid * PIECE);
    const unsigned kofs = (unsigned)t * (BK * 2);
    sfor<4>([&](auto Q) { dma16<Q * 4 * PIECE>(srdA, voA[Q], kofs, sb); });
    sfor<4>([&](auto Q) { dma16<OPI + Q * 4 * PIECE>(srdB, voB[Q], kofs, sb); });
  };

  f32x4_t acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  if (nk > 0) issue(0, 0);
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_nop 4" ::: "memory");  // zeroed accumulators -> MFMA SrcC
  __builtin_amdgcn_sched_barrier(0);
  for (int t = 0; t < nk; ++t) {
    const unsigned st = (unsigned)(t & 1) * STAGE;
    vmcnt<0>();  // this wave's DMAs of tile t landed ...
    barrier();   // ... and every wave's; every wave is done reading tile t - 1's stage
    if (t + 1 < nk) issue(t + 1, (unsigned)((t + 1) & 1));
    bf16x8_t a[2][4], b[2][4];
    // k-step 0 and 1 fragments (16 reads), MFMAs of k-step 0 behind k-step 1's reads
    sfor<4>([&](auto I) { ds16<I * 2 * PIECE>(a[0][I], rdA + st + ch0); });
    sfor<4>([&](auto J) { ds16<J * 2 * PIECE>(b[0][J], rdB + st + ch0); });
    sfor<4>([&](auto I) { ds16<I * 2 * PIECE>(a[1][I], rdA + st + ch1); });
    sfor<4>([&](auto J) { ds16<J * 2 * PIECE>(b[1][J], rdB + st + ch1); });
    lgkm<8>();
    sfor<4>([&](auto I) { tie(a[0][I]); tie(b[0][I]); });
    sfor<16>([&](auto S) {
      constexpr int i = S / 4, j = S % 4;
      mfma<E>(acc[i][j], b[0][j], a[0][i]);
    });
    lgkm<0>();
    sfor<4>([&](auto I) { tie(a[1][I]); tie(b[1][I]); });
    sfor<16>([&](auto S) {
      constexpr int i = S / 4, j = S % 4;
      mfma<E>(acc[i][j], b[1][j], a[1][i]);
    });
  }
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");  // last MFMAs -> VALU reads
  __builtin_amdgcn_sched_barrier(0);

  const int lr = lane & 15, hc = lane >> 4;  // acc row, 4-column group of the fragment
  if (p.ks > 1) {
    // split-K: this slice's fp32 partial tile, then the last arrival sums the slices
    float* wsl = p.ws + ((long)slice * ntile + tile) * (BM * BN);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int row = wm * 64 + i * 16 + lr, col = wn * 64 + j * 16 + hc * 4;
        *reinterpret_cast<f32x4_t*>(wsl + row * BN + col) = acc[i][j];
      }
    __threadfence();
    __syncthreads();
    __shared__ unsigned last;
    if (tid == 0) {
      const unsigned prev = atomicAdd(p.tickets + tile, 1u);
      last = prev == (unsigned)p.ks - 1;
      if (last) p.tickets[tile] = 0u;  // reset for the next launch (stream-ordered)
    }
    __syncthreads();
    if (!last) return;
    __threadfence();
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int row = wm * 64 + i * 16 + lr, col = wn * 64 + j * 16 + hc * 4;
        f32x4_t s = f32x4_t{0.f, 0.f, 0.f, 0.f};
        for (int k = 0; k < p.ks; ++k)  // fixed order: bit-reproducible
          s += *reinterpret_cast<const f32x4_t*>(p.ws + ((long)k * ntile + tile) * (BM * BN) + row * BN + col);
        acc[i][j] = s;
      }
  }

  // ---- epilogue through LDS: tile rows of 256 B, chunk c at c ^ (row & 15), its 8-B halves
  // exchanged in rows with bit 3 set: a 16-lane ds_write_b64 group (rows lr = 0..15) then covers
  // all 32 write banks ((a / 4) % 32) instead of 16 (as gemm_w4.h's epilogue)
  __syncthreads();  // every wave's last fragment reads are done (no DMA is in flight)
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = wm * 64 + i * 16 + lr;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int ch = wn * 8 + 2 * j + (hc >> 1);
      const f32x4_t v = acc[i][j];
      uint2 o;
      o.x = pk2<E>(v[0], v[1]);
      o.y = pk2<E>(v[2], v[3]);
      *reinterpret_cast<uint2*>(smem + row * 256 + ((ch ^ (row & 15)) << 4) + (((hc ^ (row >> 3)) & 1) << 3)) = o;
    }
  }
  __syncthreads();
  const int cc = tid & 15;
#pragma unroll 4
  for (int rr = 0; rr < 8; ++rr) {
    const int row = rr * 16 + (tid >> 4);
    uint4 v = *reinterpret_cast<const uint4*>(smem + row * 256 + ((cc ^ (row & 15)) << 4));
    if (row & 8) v = make_uint4(v.z, v.w, v.x, v.y);
    const long gm = m0 + row;
    const int gn = n0 + cc * 8;
    if constexpr (RES) {
      float a8[8], r8[8];
      unpack8e<E>(v, a8);
      unpack8e<E>(*reinterpret_cast<const uint4*>(p.r + gm * p.ldr + gn), r8);
#pragma unroll
      for (int q = 0; q < 8; ++q) a8[q] += r8[q];
      v = pack8e<E>(a8);
    }
    *reinterpret_cast<uint4*>(p.c + gm * p.ldc + gn) = v;
  }
}

// split-K factor for ks = 0: none. The in-kernel slice reduction (agent-scope release fence per
// workgroup = an L2 write-back on this chip) measured 3-5x slower than no split on the GPT-2 products
// (profiles/r3_gemm_s_vs_hipblaslt.log); ks > 1 stays available explicitly (tests cover it).
int pick_ks(long, long) { return 1; }

}  // namespace

// C = A @ B^T (+ residual): A [M, K], B [N, K]; M, N % 128, K % 64. ks = 0 picks split-K.
at::Tensor gemm_nt_s(const at::Tensor& a, const at::Tensor& b, const std::optional<at::Tensor>& out,
                     const std::optional<at::Tensor>& residual, int64_t ks) {
  FT_CHECK_CUDA(a);
  TORCH_CHECK(a.scalar_type() == at::kBFloat16 || a.scalar_type() == at::kHalf, "gemm_nt_s: bf16 / fp16");
  TORCH_CHECK(b.scalar_type() == a.scalar_type(), "gemm_nt_s: A / B dtype mismatch");
  FT_CHECK_CONTIG(a);
  FT_CHECK_CONTIG(b);
  TORCH_CHECK(a.dim() == 2 && b.dim() == 2 && a.size(1) == b.size(1), "gemm_nt_s: A [M, K], B [N, K]");
  const long M = a.size(0), K = a.size(1), N = b.size(0);
  TORCH_CHECK(M % BM == 0 && N % BN == 0 && K % BK == 0 && K >= BK, "gemm_nt_s: M, N % 128, K % 64 (got ",
              M, " ", N, " ", K, ")");
  TORCH_CHECK(M * K * 2 < (1L << 32) && N * K * 2 < (1L << 32), "gemm_nt_s: operand over 4 GiB");
  const at::DeviceGuard guard(a.device());
  at::Tensor c;
  if (out.has_value() && out->defined()) {
    c = *out;
    TORCH_CHECK(c.scalar_type() == a.scalar_type(), "gemm_nt_s: out dtype");
    FT_CHECK_CONTIG(c);
    TORCH_CHECK(c.numel() == M * N, "gemm_nt_s: out has the wrong size");
  } else {
    c = at::empty({M, N}, a.options());
  }
  SArgs p{};
  p.a = cptr<bf16_t>(a);
  p.b = cptr<bf16_t>(b);
  p.c = mptr<bf16_t>(c);
  p.lda = K;
  p.ldb = K;
  p.ldc = N;
  p.ldr = N;
  p.M = M;
  p.N = N;
  p.K = K;
  p.tiles_m = M / BM;
  p.tiles_n = N / BN;
  const long tiles = (long)p.tiles_m * p.tiles_n;
  const int kt = (int)(ks > 0 ? ks : pick_ks(tiles, K / BK));
  TORCH_CHECK(kt >= 1 && kt <= 16, "gemm_nt_s: split-K factor 1..16");
  p.ks = kt;
  at::Tensor ws, tk;
  if (kt > 1) {
    ws = at::empty({(long)kt * tiles * BM * BN}, a.options().dtype(at::kFloat));
    // per-tile tickets, zeroed once per launch (the kernel also resets them after use)
    tk = at::zeros({tiles}, a.options().dtype(at::kInt));
    p.ws = mptr<float>(ws);
    p.tickets = reinterpret_cast<unsigned*>(tk.data_ptr<int>());
  }
  bool res = false;
  if (residual.has_value() && residual->defined()) {
    TORCH_CHECK(residual->scalar_type() == a.scalar_type(), "gemm_nt_s: residual dtype");
    FT_CHECK_CONTIG((*residual));
    TORCH_CHECK(residual->numel() == M * N, "gemm_nt_s: residual has the wrong size");
    p.r = cptr<bf16_t>(*residual);
    res = true;
  }
  const dim3 grid((unsigned)(tiles * kt));
  FT_DISPATCH_E16(a.scalar_type(), {
    if (res)
      hipLaunchKernelGGL((gemm_s_kernel<E, true>), grid, dim3(NT), 0, ft_stream(), p);
    else
      hipLaunchKernelGGL((gemm_s_kernel<E, false>), grid, dim3(NT), 0, ft_stream(), p);
  });
  FT_LAUNCH_CHECK();
  return c;
}

TORCH_LIBRARY_FRAGMENT(ftamd, m) {
  m.def("gemm_nt_s(Tensor a, Tensor b, Tensor(a!)? out=None, Tensor? residual=None, int ks=0) -> Tensor",
        &gemm_nt_s);
}
