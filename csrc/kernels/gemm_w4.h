// 4-wave bf16 / fp16 GEMM for gfx950 with an instruction-level schedule (the "w4" kernel).
//
//   C[M, N] = sum_k A(m, k) * B(k, n)
//   A: K-contiguous  A(m, k) = a[m * lda + k]   (activations x [T, K]; dY [T, N] of a dX)
//      k-major (AT)  A(m, k) = a[k * lda + m]   (dY^T of a weight gradient: dY is [T, N], m = n)
//   B: K-contiguous  B(k, n) = b[n * ldb + k]   (nn.Linear weight [N, K]: every forward)
//      k-major (BT)  B(k, n) = b[k * ldb + n]   (weight [N, K] read as K x N in dX; X [T, K] in dW)
// so every product of the transformer step reads its operands as they are stored (reference
// model.py:195,215,254,379 forward; their dX = dY W and dW = dY^T X backward): no transposed
// copies, no separate transpose kernel.
//
// Structure (one workgroup = one 256 x BN output tile, BN = 32 * NJ, BK = 64):
//   * 4 waves, one per SIMD, each owning a 128 x (16 NJ) quadrant = 8 x NJ fragments of
//     v_mfma_f32_16x16x32_bf16 (_f16 for --model-dtype fp16); the accumulators are pinned in AGPRs (the MFMAs are inline asm on
//     "+a" operands, so the compiler never shuffles them), the operand fragments in VGPRs.
//     NJ is chosen per shape so the tile count fills the 256 CUs in whole rounds (the 8B step:
//     qkv 256 x 192 -> 256 tiles, w13 256 x 224 -> 4 x 256, wo / w2 256 x 128 -> 256, head 256^2).
//   * Both operands are staged by LDS-DMA (buffer_load_dwordx4 ... lds: 1 KiB per wave-instruction,
//     no staging VGPRs, the per-lane SOURCE offset carries the swizzle), double-buffered (2 stages
//     of 32 + 4 NJ KiB). Two image kinds:
//       K-contiguous: [rows][64 k], 128-B rows, 16-B chunk c of row r at c ^ (r & 7): the
//         fragment is one ds_read_b128 (8 consecutive k of one row), conflict-free.
//       k-major: [64 k][cols], rows of 2 x cols bytes, read with ds_read_b64_tr_b16 (the hardware
//         transpose: a 16-lane group gets 4 k-rows x 16 columns column-major, so two reads give the
//         same 8-consecutive-k fragment as ds_read_b128 — the two kinds mix freely). The 32-B
//         column pair j of k-row k sits at pair j ^ sigma(k), sigma chosen per row length so the
//         8 rows one 32-lane half reads (k .. k+3, k+8 .. k+11) hit 8 distinct 8-bank windows
//         (conflict-free); sigma depends on k only through bits the k-step / hi-half offsets never
//         change, so each fragment needs ONE lane address and the rest are immediates.
//   * One K-tile = 2 x 8 NJ MFMAs per wave (two k-steps of 32). The fragment registers are
//     double-buffered by k-step, so every LDS read is issued right behind an MFMA and consumed a
//     k-step later:
//       MFMA 0 .. RS-1 : the k-step-1 fragment reads of this tile (R read instructions, RPS per MFMA)
//       MFMA SB1       : lgkmcnt(0) + barrier  -> every wave has finished reading this stage
//       then           : the 8 + NJ LDS-DMAs of tile t+2 into this stage, spread evenly
//       MFMA SB2       : vmcnt(8 + NJ) + barrier -> tile t+1 (issued one K-tile ago) has landed
//       then           : the k-step-0 fragment reads of tile t+1
//     This is the counts-and-placement schedule of the vendor's tuned assembly GEMMs on this chip
//     (one wave per SIMD, direct-to-LDS, prefetch two tiles ahead), with HIP choosing registers.
//   * Epilogue through LDS: per-lane stores straight from the MFMA accumulator layout write 16
//     rows x 32 B per instruction and cost 20-26 % of the kernel (ablation in
//     profiles/r3_gemm_w4_investigation.md); each wave instead parks its quadrant in 32 KiB of the
//     idle LDS (256-B rows, 16-B chunks XOR-swizzled by row: conflict-free 8-B writes and 16-B
//     row reads) and stores whole rows, 4 x 256 B per instruction. Fused epilogues act on the
//     row-contiguous values: + residual / accumulate (wo / w2 into the residual stream, gradient
//     accumulation), RoPE on the packed Q/K columns of the QKV projection (reference
//     model.py:100-126), SwiGLU forward (model.py:254) and backward (dX of w2 -> dgu from the
//     saved gu), and the per-tile sum of squares of a weight gradient (clip_grad_norm_'s
//     input, reference utils.py:58-63) so no separate pass re-reads the gradient.
//   * Tiles are mapped XCD-contiguously (blockIdx % 8 = XCD under round-robin dispatch), rastered
//     so that the larger operand's panels stay inside one XCD's L2 (M-fastest when B is larger).
#pragma once

#include "torch_utils.h"

#include <utility>

namespace ftw4 {


typedef int i32x4_t __attribute__((ext_vector_type(4)));

template <typename F, int... I>
__device__ __forceinline__ void sfor_impl(F&& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, typename F>
__device__ __forceinline__ void sfor(F&& f) {
  sfor_impl(f, std::make_integer_sequence<int, N>{});
}

constexpr int BM = 256, BK = 64, NT = 256;
constexpr int PIECE = 1024;  // one LDS-DMA wave-instruction: 8 image rows of 128 B
constexpr int FS = 2 * PIECE;  // one 16-row fragment (K-contiguous image)
constexpr int OPA = 32 * PIECE;  // A image: 256 rows x 64 k
constexpr int RBA = 2 * BM;      // k-major A image: 512-B k-rows

enum W4Epi : int { W4_STORE = 0, W4_RES = 1, W4_ROPE = 2, W4_SWIGLU = 3, W4_SWIGLU_BWD = 4 };

__device__ __forceinline__ unsigned lds_u32(const void* p) {
  return (unsigned)(uintptr_t)((const __attribute__((address_space(3))) char*)p);
}

// raw buffer resource over [p, p + 4 GiB): stride 0, num_records = max, gfx9 default format
__device__ __forceinline__ i32x4_t make_srd(const void* p) {
  const unsigned long long a = (unsigned long long)p;
  i32x4_t r;
  r[0] = __builtin_amdgcn_readfirstlane((int)(unsigned)a);
  r[1] = __builtin_amdgcn_readfirstlane((int)((unsigned)(a >> 32) & 0xffffu));
  r[2] = -1;
  r[3] = 0x00020000;
  return r;
}

// LDS-DMA, 2 instructions: 16 B per lane from srd + voff + soff into LDS [m0 + 16 * lane],
// m0 = sbase + IMM. m0 is used by nothing else in this kernel (no LDS-DMA builtins, no GDS), so it
// is not saved; gfx950 needs no wait state between the m0 write and the DMA. s_add_u32 writes SCC:
// declared, else the scheduler may put the K loop's compare before a DMA and branch on the carry.
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

template <int OFF>
__device__ __forceinline__ void dstr(bf16x4_t& d, unsigned addr) {
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(d) : "v"(addr), "i"(OFF) : "memory");
}

// bf16 or fp16 operands (--model-dtype): same shape, same schedule, another opcode
template <class E>
__device__ __forceinline__ void mfma(f32x4_t& c, const bf16x8_t& a, const bf16x8_t& b) {
  if constexpr (std::is_same<E, EF16>::value)
    asm volatile("v_mfma_f32_16x16x32_f16 %0, %1, %2, %0" : "+a"(c) : "v"(a), "v"(b));
  else
    asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(c) : "v"(a), "v"(b));
}

template <int N>
__device__ __forceinline__ void lgkm() {
  asm volatile("s_waitcnt lgkmcnt(%0)" ::"i"(N < 15 ? N : 15) : "memory");
}
template <int N>
__device__ __forceinline__ void vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"i"(N) : "memory");
}
__device__ __forceinline__ void barrier() { asm volatile("s_barrier" ::: "memory"); }
// an epilogue staging chunk with its 8-B halves exchanged when s (rows with bit 3 set; see the
// epilogue): the same call converts either way
__device__ __forceinline__ uint4 stg_swap(uint4 v, bool s) {
  return s ? make_uint4(v.z, v.w, v.x, v.y) : v;
}

// ---- fragments: one 128-bit register (ds_read_b128) or two 64-bit halves (two tr reads) ------
template <bool T>
struct Frag;
template <>
struct Frag<false> {
  bf16x8_t v;
};
template <>
struct Frag<true> {
  bf16x4_t lo, hi;
};
__device__ __forceinline__ bf16x8_t val(const Frag<false>& f) { return f.v; }
__device__ __forceinline__ bf16x8_t val(const Frag<true>& f) {
  return __builtin_shufflevector(f.lo, f.hi, 0, 1, 2, 3, 4, 5, 6, 7);
}
// the registers an asm wait covered: consumers stay behind the wait
__device__ __forceinline__ void tie(Frag<false>& x) { asm volatile("" : "+v"(x.v)); }
__device__ __forceinline__ void tie(Frag<true>& x) {
  asm volatile("" : "+v"(x.lo));
  asm volatile("" : "+v"(x.hi));
}

// XOR applied to the 32-B column-pair index of k-row k in a k-major image with RB-byte rows.
// A 32-lane half of a transposed read takes rows k0 + {0..3, 8..11} (4 lanes x 8 B = one pair per
// row): they must land in 8 distinct 8-dword bank windows. Row r's pair p is window
// (r * RB / 32 + (p ^ sigma(r))) mod 8.
template <int RB>
__device__ __forceinline__ int tsw(int k) {
  if constexpr (RB % 256 == 0)  // every row starts in window 0: spread rows over all 8
    return (k & 3) | (((k >> 3) & 1) << 2);
  else if constexpr (RB == 448)  // rows 0..3 -> windows 0, 6, 4, 2 already; 8..11 onto the odd ones
    return (k >> 3) & 1;
  else if constexpr (RB == 384)  // rows alternate windows 0 / 4: pairs ^ 0..3 fill the rest
    return ((k >> 1) & 1) | (((k >> 3) & 1) << 1);
  else
    static_assert(RB % 256 == 0 || RB == 448 || RB == 384, "k-major image row length");
  return 0;
}

struct W4Args {
  const bf16_t* a;
  const bf16_t* b;
  bf16_t* c;
  const bf16_t* r;       // residual (may alias c: accumulate) or null; W4_SWIGLU_BWD: gu
  const float* cos_t;    // RoPE: [S, D/2] tables
  const float* sin_t;
  float* part;           // per-tile sums of squares of the stored C (null: none)
  int part_n;            // slots in part: the ones past tiles_m * tiles_n are zeroed (workgroup 0)
  long lda, ldb, ldc, ldr;
  int M, N, K;
  int tiles_m, tiles_n;
  int nfast;             // raster N-fastest inside an XCD's range (A is the larger operand)
  int group;             // > 1: grouped raster, bands of `group` slow-dimension tiles (tile_of)
  int rope_cols;         // RoPE: columns [0, rope_cols) are rotated (Hq + Hkv heads)
  int rope_hd;           // head dim
  int rope_seq;          // sequence length (position = row % seq)
  // SwiGLU epilogue (W4_SWIGLU): b = [w1; w3] ([2F, K]); tile tn covers features
  // [tn * 16 NJ, +16 NJ) of BOTH halves (B image rows = that slice of w1, then of w3), so the
  // tile holds g and u of the same features: c = gu [M, 2F], a = silu(g) u [M, F], a^T [F, M]
  // W4_SWIGLU_BWD: the tile is da [M, F] (dX of w2); c = dgu [M, 2F] from r = gu [M, 2F]
  int ffn;               // F
  bf16_t* act;           // a
  bf16_t* actT;          // a^T (null: not written)
  int exact;             // IEEE division in the sigmoid (FT_EXACT_MATH), as swiglu_fwd_t
  // split-K (W4_STORE / W4_RES, K-contiguous A): splits = S in 2 .. 8 runs each output tile as
  // S workgroups over S slices of K (grid = S x tiles, slice-major). Slices 0 .. S-2 park their
  // fp32 accumulators in ws (fragment order: [tile][slice][wave][i][j][lane] float4, 1 KiB per
  // wave store) and raise flag tick[8 tile + slice]; the last slice adds them in slice order to
  // its own in the epilogue (fixed order: deterministic) and re-arms the flags for the next launch.
  int splits;
  int dbg;               // timing probes only (gemm_w4_set_dbg): bit 0 = skip the epilogue's global stores;
                         // bit 1 (tests): split-K producers never raise their flags (the timeout path)
  long long* prof;       // timing probe (gemm_w4_set_prof; scripts/w4_timeline.py): [grid][8] int64
  int* tick;             // [8 * tiles] int32, zero between launches (per device and stream)
  float* ws;             // [tiles * (S - 1) * 256 * BN] fp32
  // split-K hand-off that never completed (a producer lost, > spin polls): the consumer adds 1 to
  // *err (read by gemm_w4_splitk_errors), writes NaN for the whole tile (so the step's non-finite
  // guard skips the update and the trainer stops on it) and re-arms only the flags it saw raised
  int* err;
  int spin;              // consumer poll bound (2^22 ~ seconds; tests lower it)
  int deadzero;          // the last two K-tiles' DMAs read nothing (null descriptor; gemm_w4_set_deadzero)
};

// (tm, tn) of workgroup bid (returned by value: through references the pair went to scratch)
// Workgroup bid runs on XCD bid % 8 (round-robin dispatch); each XCD takes a contiguous range w of
// the raster, so the tiles one XCD runs together share operand panels in its L2. group > 1: the
// raster sweeps bands of `group` slow-dimension tiles (the XCD's 32 concurrent tiles then form a
// group x 32/group block: fewer distinct panels per K-step than a 1- or 2-row strip).
__device__ __forceinline__ int2 tile_of(int bid, int tiles_m, int tiles_n, int nfast, int group) {
  const int nwg = tiles_m * tiles_n;
  const int q = nwg / 8, rem = nwg % 8;
  const int x = bid % 8, o = bid / 8;
  const int w = (x < rem ? x * (q + 1) : rem * (q + 1) + (x - rem) * q) + o;
  if (group > 1) {
    if (nfast) {
      const int band = group * tiles_n, g = w / band, r = w - g * band;
      const int gm = min(group, tiles_m - g * group);
      return make_int2(g * group + r % gm, r / gm);
    }
    const int band = group * tiles_m, g = w / band, r = w - g * band;
    const int gn = min(group, tiles_n - g * group);
    return make_int2(r / gn, g * group + r % gn);
  }
  return nfast ? make_int2(w / tiles_n, w % tiles_n) : make_int2(w % tiles_m, w / tiles_m);
}

// the accumulators "written" by an empty asm: a point the register allocator's copies and
// materialisations of them cannot cross (see the uses)
template <int NJ>
__device__ __forceinline__ void tie_acc(f32x4_t (&acc)[8][NJ]) {
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) asm volatile("" : "+a"(acc[i][j]));
}

template <int NJ, bool AT, bool BT>
struct Frags {
  Frag<AT> a0[8], a1[8];
  Frag<BT> b0[NJ], b1[NJ];
};

__device__ __forceinline__ void tie_frag(Frag<false>& x) { asm volatile("" : "+v"(x.v)); }
__device__ __forceinline__ void tie_frag(Frag<true>& x) { asm volatile("" : "+v"(x.lo), "+v"(x.hi)); }

// every fragment register "written" here: the asm LDS reads are asynchronous, but the compiler
// takes their outputs as complete at the asm, so it may hand a register whose read is still in
// flight (the dead next-k-step reads of the last K-tile) to other code; a tie placed after the
// lgkmcnt(0) wait keeps all of them reserved until the reads have landed
template <int NJ, bool AT, bool BT>
__device__ __forceinline__ void tie_frags(Frags<NJ, AT, BT>& f) {
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    tie_frag(f.a0[i]);
    tie_frag(f.a1[i]);
  }
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    tie_frag(f.b0[j]);
    tie_frag(f.b1[j]);
  }
}

template <int NJ, bool AT, bool BT>
struct Sched {
  static constexpr int MH = 8 * NJ;          // MFMAs per k-step
  static constexpr int NA = AT ? 2 : 1;      // read instructions per A / B fragment
  static constexpr int NB = BT ? 2 : 1;
  static constexpr int R = 8 * NA + NJ * NB; // read instructions per k-step: b[0], a[0..7], b[1..]
  static constexpr int F1 = NB + 8 * NA;     // ... of which the first MFMA run needs these
  static constexpr int D = 8 + NJ;           // LDS-DMAs per wave per K-tile (A 8, B NJ)
  static constexpr int RB = 64 * NJ;         // k-major B image row bytes
  static constexpr int fits(int rps) {
    return (2 * MH - (R + rps - 1) / rps - 4) - ((R + rps - 1) / rps + 8 > 24 ? (R + rps - 1) / rps + 8 : 24) - 4 >= D;
  }
  static constexpr int RPS = fits(1) ? 1 : 2;  // read instructions per MFMA slot
  static constexpr int RS = (R + RPS - 1) / RPS;  // MFMA slots the reads of one k-step take
  static constexpr int SB1 = RS + 8 > 24 ? RS + 8 : 24;  // first barrier (after MFMA SB1)
  static constexpr int SB2 = 2 * MH - RS - 4;  // second barrier
  static constexpr int dma_slot(int d) { return SB1 + 2 + d * (SB2 - SB1 - 4) / D; }
  static constexpr int OPB = NJ * 4 * PIECE;  // B image
  static constexpr int ST = OPA + OPB;        // stage
  // LDS: A stage 0 | A stage 1 | B stage 0 | B stage 1, so a stage's offset (32 KiB for A, 4 NJ
  // KiB for B) plus every fragment / k-step / half offset fits the 16-bit DS immediate: with the
  // K-tile loop unrolled by two, no fragment read needs an address add
  static constexpr int A_AT(int st) { return st * OPA; }
  static constexpr int B_AT(int st) { return 2 * OPA + st * OPB; }
  static constexpr int B_RD(int st) { return st * OPB; }  // B read bases already hold 2 * OPA
  static_assert(SB2 - SB1 - 4 >= D && SB2 + RS < 2 * MH, "schedule does not fit");
  // largest DS immediates: stage 1 + k-step 1 + hi half / last fragment (16-bit offset field)
  static_assert(OPA + 32 * RBA + 4 * RBA < 65536 && OPA + FS * 7 < 65536, "A read offset");
  static_assert(OPB + 32 * RB + 4 * RB < 65536 && OPB + FS * (NJ - 1) < 65536, "B read offset");
};

struct Ctx {
  i32x4_t srdA, srdB;
  i32x4_t srdA0, srdB0;             // same bases, num_records 0: every load out of range (zeros, no traffic)
  unsigned voA[8], voB[8];
  unsigned rdA0, rdA1, rdB0, rdB1;  // K-contiguous images: k-step 0 / 1 lane address
  unsigned aT[8], bT[8];            // k-major images: lane address of fragment i (k-step 0, lo)
  unsigned lds0;
  unsigned sbase;                   // LDS-DMA: this wave's first piece (m0 base, SGPR)
  unsigned stepA, stepB;            // bytes one K-tile advances the A / B source
  int wid;
};

// read instruction r (b[0], a[0..7], b[1..NJ-1]; a k-major fragment is two: lo, hi) of k-step KK
// from stage ST (lane base address + immediate)
template <int NJ, bool AT, bool BT, int KK, int ST, int r>
__device__ __forceinline__ void rd(Frag<AT> (&ax)[8], Frag<BT> (&bx)[NJ], const Ctx& c) {
  using S = Sched<NJ, AT, BT>;
  constexpr int NA = S::NA, NB = S::NB;
  constexpr bool isA = r >= NB && r < NB + 8 * NA;
  if constexpr (isA) {
    constexpr int i = (r - NB) / NA, h = (r - NB) % NA;
    if constexpr (AT) {
      if constexpr (h == 0)
        dstr<S::A_AT(ST) + KK * 32 * RBA>(ax[i].lo, c.aT[i]);
      else
        dstr<S::A_AT(ST) + KK * 32 * RBA + 4 * RBA>(ax[i].hi, c.aT[i]);
    } else {
      ds16<S::A_AT(ST) + FS * i>(ax[i].v, KK ? c.rdA1 : c.rdA0);
    }
  } else {
    constexpr int j = r < NB ? 0 : 1 + (r - NB - 8 * NA) / NB;
    constexpr int h = r < NB ? r : (r - NB - 8 * NA) % NB;
    if constexpr (BT) {
      constexpr int RB = S::RB;
      if constexpr (h == 0)
        dstr<S::B_RD(ST) + KK * 32 * RB>(bx[j].lo, c.bT[j]);
      else
        dstr<S::B_RD(ST) + KK * 32 * RB + 4 * RB>(bx[j].hi, c.bT[j]);
    } else {
      ds16<S::B_RD(ST) + FS * j>(bx[j].v, KK ? c.rdB1 : c.rdB0);
    }
  }
}

// the reads of MFMA slot `slot` (RPS instructions) of k-step KK
template <int NJ, bool AT, bool BT, int KK, int ST, int slot>
__device__ __forceinline__ void rd_slot(Frag<AT> (&ax)[8], Frag<BT> (&bx)[NJ], const Ctx& c) {
  using S = Sched<NJ, AT, BT>;
  sfor<S::RPS>([&](auto QQ) {
    constexpr int r = slot * S::RPS + QQ;
    if constexpr (r < S::R) rd<NJ, AT, BT, KK, ST, r>(ax, bx, c);
  });
}

// One K-tile t in stage CUR = t & 1: DMA: stage tile t + 2 into this stage (clamped to the last
// tile: the last two K-tiles re-stage it into a stage nobody reads again); NEXT: read tile t + 1's
// first k-step (stage 1 - CUR; after the last tile these reads are dead).
template <class E, int NJ, bool AT, bool BT, int CUR, bool DMA, bool NEXT>
__device__ __forceinline__ void ktile(f32x4_t (&acc)[8][NJ], Frags<NJ, AT, BT>& f, int t, int nk, const Ctx& c) {
  using S = Sched<NJ, AT, BT>;
  // the last two K-tiles have no tile t + 2: their DMAs go through the null descriptors (every load
  // out of range: zeros into the dead stage, no memory request, nothing for the drain's vmcnt(0) to
  // wait on) -- before round 6 they re-staged the last tile from L2 (W4Args::deadzero = 0)
  const bool live = t + 2 < nk;
  const int tn2 = __builtin_amdgcn_readfirstlane(min(t + 2, nk - 1));
  const unsigned kofsA = (unsigned)tn2 * c.stepA, kofsB = (unsigned)tn2 * c.stepB;
  const i32x4_t dsrdA = live ? c.srdA : c.srdA0, dsrdB = live ? c.srdB : c.srdB0;
  const unsigned sb = c.sbase;
  sfor<2 * S::MH>([&](auto SS) {
    constexpr int s = SS;
    constexpr int i = s & 7, j = (s % S::MH) >> 3;  // runs of 8 MFMAs share the B fragment (SrcA)
    if constexpr (s == 0) {  // the first run's fragments landed (issued last K-tile)
      lgkm<S::R - S::F1>();
      tie(f.b0[0]);
      sfor<8>([&](auto I) { tie(f.a0[I]); });
    }
    if constexpr (s == 8) {  // all of k-step 0 (the k-step-1 reads of slots 0..7 in flight)
      lgkm<8 * S::RPS>();
      sfor<NJ>([&](auto J) { tie(f.b0[J]); });
    }
    if constexpr (s == 2) asm volatile("s_setprio 3" ::: "memory");
    if constexpr (s < S::MH)
      mfma<E>(acc[i][j], val(f.b0[j]), val(f.a0[i]));
    else
      mfma<E>(acc[i][j], val(f.b1[j]), val(f.a1[i]));
    if constexpr (s < S::RS) rd_slot<NJ, AT, BT, 1, CUR, s>(f.a1, f.b1, c);
    if constexpr (s == S::SB1) {  // this stage fully read by every wave -> it may be restaged
      lgkm<0>();
      sfor<8>([&](auto I) { tie(f.a1[I]); });
      sfor<NJ>([&](auto J) { tie(f.b1[J]); });
      barrier();
    }
    if constexpr (DMA) {
      sfor<S::D>([&](auto DD) {
        constexpr int d = DD;
        if constexpr (s == S::dma_slot(d)) {
          // interleave A and B pieces: even slots A (while any), odd slots B
          constexpr int qa = d < 2 * NJ ? d / 2 : NJ + (d - 2 * NJ);
          constexpr bool isA = d < 2 * NJ ? (d % 2 == 0) : true;
          if constexpr (isA)
            dma16<S::A_AT(CUR) + qa * 4 * PIECE>(dsrdA, c.voA[qa], kofsA, sb);
          else
            dma16<S::B_AT(CUR) + (d / 2) * 4 * PIECE>(dsrdB, c.voB[d / 2], kofsB, sb);
        }
      });
    }
    if constexpr (s == S::SB2 - 1) asm volatile("s_setprio 0" ::: "memory");
    if constexpr (NEXT && s == S::SB2) {  // tile t + 1 landed (this K-tile's DMAs stay in flight)
      if constexpr (DMA)
        vmcnt<S::D>();
      else
        vmcnt<0>();
      barrier();
    }
    if constexpr (NEXT && s > S::SB2 && s <= S::SB2 + S::RS) rd_slot<NJ, AT, BT, 0, 1 - CUR, s - S::SB2 - 1>(f.a0, f.b0, c);
    if constexpr (s == 2 * S::MH - 1) asm volatile("s_setprio 0" ::: "memory");
  });
}

template <class E, int NJ, int EPI, bool AT, bool BT>
__global__ __launch_bounds__(NT, 1) void gemm_w4_kernel(W4Args p) {
  using S = Sched<NJ, AT, BT>;
  constexpr int LDS = 2 * S::ST > 4 * 32768 ? 2 * S::ST : 4 * 32768;  // stages / epilogue staging
  __shared__ __attribute__((aligned(1024))) char smem[LDS];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  // timing probe: exit stamp (probe_end). (Any stamp before the drain - even one stored at entry,
  // older than every DMA - made the compiler move address clamps into the dW K loops: the static
  // check rejects such builds.) The investigation build (-DFT_W4_PROBE, scripts/w4_probe_build.py:
  // a separate library loaded through FT_KERNELS_SO, not statically checked) also stamps the entry,
  // the end of the prologue, the drain and the end of the epilogue's LDS staging.
#ifdef FT_W4_PROBE
  long long pt0 = __builtin_amdgcn_s_memrealtime(), pt1 = 0, pt2 = 0, pt3 = 0;
#endif
  const int wm = wid >> 1, wn = wid & 1;
  constexpr int BN = 32 * NJ, NW = 16 * NJ;
  const int ntiles = p.tiles_m * p.tiles_n;
  const int nsplit = p.splits > 1 ? p.splits : 1;
  const int ks = blockIdx.x / ntiles;        // K slice of a split-K tile (0 without split)
  const int tb = blockIdx.x - ks * ntiles;   // output tile
  const int2 tt = tile_of(tb, p.tiles_m, p.tiles_n, p.nfast, p.group);
  const int tm = tt.x, tn = tt.y;
  const int m0 = tm * BM, n0 = tn * BN;
  const int f0 = tn * NW;  // W4_SWIGLU: first feature of the tile (NW features of w1 and of w3)
  // K-tiles in pairs; slice ks takes pairs [np * ks / S, np * (ks + 1) / S) (host: np >= S)
  const int npairs = p.K / (2 * BK);
  const int kp0 = npairs * ks / nsplit, kp1 = npairs * (ks + 1) / nsplit;
  const int nk = 2 * (kp1 - kp0);            // K-tiles of this workgroup (even)
  const long k0 = (long)kp0 * 2 * BK;        // its first k

  // LDS-DMA sources. Instruction q of wave w fills image piece P = q * 4 + w (bytes [P KiB, +1 KiB)),
  // lane L its 16 B at P KiB + 16 L; the lane's source is the element that image slot holds.
  // A tail tile of the dW layout (M % 256: the GPT-2 LM-head dW, M = V = 50304) clamps the sources of
  // its rows past M onto the last 8-row chunk (k-major A, M % 8): every load stays inside A, and
  // those rows' results are never stored. (The other layouts take M % 256: no clamp, no guard.)
  const int mlast = min(BM, p.M - m0) - 1;  // last valid tile row
  const bool mtail = AT && m0 + BM > p.M;   // uniform
  Ctx c;
  c.wid = wid;
  c.lds0 = __builtin_amdgcn_readfirstlane(lds_u32(smem));
  const int lrow = wid * 8 + (lane >> 3), lch = (lane & 7) ^ (lane >> 3);
  if constexpr (AT) {
    // [64 k][256 m], 512-B rows: piece P holds k-rows 2P, 2P + 1
    c.srdA = make_srd(p.a + m0 + k0 * p.lda);
    c.stepA = (unsigned)(BK * p.lda * 2);
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int off = (q * 4 + wid) * PIECE + lane * 16;
      const int k = off / RBA, cp = (off % RBA) >> 4;
      const int gc = cp ^ (2 * tsw<RBA>(k));
      c.voA[q] = (unsigned)(((long)k * p.lda + min(gc * 8, mlast - 7)) * 2);
    }
  } else {
    // [256 rows][64 k], 128-B rows: lane's 16-B chunk (lane & 7) holds global chunk (lane & 7) ^ (row & 7)
    c.srdA = make_srd(p.a + (long)m0 * p.lda + k0);
    c.stepA = (unsigned)(BK * 2);
#pragma unroll
    for (int q = 0; q < 8; ++q) c.voA[q] = (unsigned)(((q * 32 + lrow) * p.lda + lch * 8) * 2);
  }
  if constexpr (BT) {
    c.srdB = make_srd(p.b + n0 + k0 * p.ldb);
    c.stepB = (unsigned)(BK * p.ldb * 2);
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int off = (q * 4 + wid) * PIECE + lane * 16;
      const int k = off / S::RB, cp = (off % S::RB) >> 4;
      const int gc = cp ^ (2 * tsw<S::RB>(k));
      c.voB[q] = (unsigned)(((long)k * p.ldb + gc * 8) * 2);
    }
  } else {
    c.srdB = make_srd((EPI == W4_SWIGLU ? p.b : p.b + (long)n0 * p.ldb) + k0);
    c.stepB = (unsigned)(BK * 2);
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int r = q * 32 + lrow;  // B image row
      const long src = EPI == W4_SWIGLU ? (r < 16 * NJ ? f0 + r : (long)p.ffn + f0 + (r - 16 * NJ)) : r;
      c.voB[q] = (unsigned)((src * p.ldb + lch * 8) * 2);
    }
  }
  c.srdA0 = c.srdA;
  c.srdB0 = c.srdB;
  if (p.deadzero) {
    c.srdA0[2] = 0;
    c.srdB0[2] = 0;
  }
  // fragment reads, K-contiguous: lane reads row r0 + (lane & 15), chunk (kk * 4 + (lane >> 4)) ^ (lane & 7)
  const unsigned lrowb = (unsigned)(((lane & 15) >> 3) * PIECE + (lane & 7) * 128);
  const unsigned lpart0 = lrowb + (unsigned)((((lane >> 4)) ^ (lane & 7)) << 4);
  const unsigned lpart1 = lrowb + (unsigned)(((4 + (lane >> 4)) ^ (lane & 7)) << 4);
  c.rdA0 = c.lds0 + wm * 16 * PIECE + lpart0;
  c.rdA1 = c.lds0 + wm * 16 * PIECE + lpart1;
  c.rdB0 = c.lds0 + 2 * OPA + wn * NJ * 2 * PIECE + lpart0;  // + S::B_RD(stage) as immediate
  c.rdB1 = c.lds0 + 2 * OPA + wn * NJ * 2 * PIECE + lpart1;
  // fragment reads, k-major: lane 4q + p of 16-lane group g supplies k-row 8 g + q (k-step 0,
  // lo half), columns 4p .. 4p + 3 of the fragment's 16 (byte 8 p of its 32-B pair)
  {
    const int g = lane >> 4, q4 = (lane & 15) >> 2, pp = lane & 3;
    const int k0 = 8 * g + q4;
    if constexpr (AT) {
      const int sg = tsw<RBA>(k0);
#pragma unroll
      for (int i = 0; i < 8; ++i)
        c.aT[i] = c.lds0 + (unsigned)(k0 * RBA + 32 * ((8 * wm + i) ^ sg) + 8 * pp);
    }
    if constexpr (BT) {
      const int sg = tsw<S::RB>(k0);
#pragma unroll
      for (int j = 0; j < NJ; ++j)
        c.bT[j] = c.lds0 + (unsigned)(2 * OPA + k0 * S::RB + 32 * ((wn * NJ + j) ^ sg) + 8 * pp);
    }
  }

  f32x4_t acc[8][NJ];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  Frags<NJ, AT, BT> f;

  // prologue: tiles 0 and 1 in flight, then tile 0's k-step-0 fragments
  c.sbase = __builtin_amdgcn_readfirstlane(c.lds0 + wid * PIECE);
  const unsigned sb = c.sbase;
  sfor<8>([&](auto Q) { dma16<S::A_AT(0) + Q * 4 * PIECE>(c.srdA, c.voA[Q], 0u, sb); });
  sfor<NJ>([&](auto Q) { dma16<S::B_AT(0) + Q * 4 * PIECE>(c.srdB, c.voB[Q], 0u, sb); });
  sfor<8>([&](auto Q) { dma16<S::A_AT(1) + Q * 4 * PIECE>(c.srdA, c.voA[Q], c.stepA, sb); });
  sfor<NJ>([&](auto Q) { dma16<S::B_AT(1) + Q * 4 * PIECE>(c.srdB, c.voB[Q], c.stepB, sb); });
  vmcnt<S::D>();
  barrier();
#ifdef FT_W4_PROBE
  pt1 = __builtin_amdgcn_s_memrealtime();
#endif
  sfor<S::R>([&](auto RR) { rd<NJ, AT, BT, 0, 0, RR>(f.a0, f.b0, c); });

  // the zeroed accumulators are MFMA sources next (VALU write -> MFMA SrcC wait states): the
  // ties pin every zero write before the pad (the register allocator places copies and
  // materialisations freely; an asm that "writes" the accumulators is a fence it cannot cross)
  tie_acc(acc);
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_nop 4" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
  // nk is even (K % 128, checked on the host): K-tiles in pairs so every stage offset is static,
  // and ONE code path for every tile (the last two re-stage the last tile and read a dead next
  // k-step): with a separate tail the register allocator placed the accumulators differently in
  // the tail and copied them across with v_accvgpr_mov right behind the asm MFMAs that were still
  // writing them (the compiler cannot see those as MFMAs) -> stale accumulators.
  int t = 0;
  do {
    ktile<E, NJ, AT, BT, 0, true, true>(acc, f, t, nk, c);
    ktile<E, NJ, AT, BT, 1, true, true>(acc, f, t + 1, nk, c);
    t += 2;
  } while (t < nk);
  // Drain: the re-staging DMAs of the last two K-tiles and the dead next-k-step reads land, and
  // the last MFMAs finish before VALU reads the accumulators (the compiler does not see the asm
  // as MFMAs, so it inserts no wait states; sched_barrier: register-only instructions may
  // otherwise be hoisted above an asm).
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
  // ... and the ties: the accumulators and fragments are (as far as the compiler knows) produced
  // here, so no read or copy of an accumulator, and no reuse of a fragment register, can be
  // placed above the drain (both happened at the loop exit without them: accumulators copied
  // right behind the asm MFMAs still writing them; index math written into registers whose
  // dead LDS reads had not returned yet)
  tie_frags(f);
  tie_acc(acc);
#ifdef FT_W4_PROBE
  pt2 = __builtin_amdgcn_s_memrealtime();
#endif
  auto probe_end = [&]() {
    if (p.prof == nullptr) return;
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    if (tid == 0) {
      unsigned hw, xcc;
      asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
      asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
      long long* r = p.prof + (long)blockIdx.x * 8;
      r[3] = __builtin_amdgcn_s_memrealtime();
      r[4] = hw;
      r[5] = xcc;
      r[6] = tb;
      r[7] = nk;
#ifdef FT_W4_PROBE
      r[0] = pt0;
      r[1] = pt1;
      r[2] = pt2;
      r[7] = pt3;
#endif
    }
  };

  // (the dW layout, k-major A, splits only its narrow tile: the GPT-2-sized weight gradients, whose
  // 18-96-tile grids cannot fill 256 CUs; the 8B grids fill the chip unsplit)
  const float4* split_slot = nullptr;  // split-K consumer: slice 0's partial (uniform)
  int split_lost = 0;                  // ... and its hand-off timed out: the tile is written as NaN
  if constexpr ((EPI == W4_STORE || EPI == W4_RES) && (!AT || NJ <= 4)) {
    if (nsplit > 1) {  // uniform (2 .. 8: host-checked)
      // Static roles, wave-uniform control flow (no single-lane branches near the 256 live
      // accumulators: those made the compiler copy them to VGPRs and spill): slices 0 .. S-2 (the
      // lower block ids: dispatched first) park their partials and raise their flags; the last
      // slice waits for all of them and adds them in slice order in its epilogue (fixed order:
      // deterministic). A waiting workgroup never holds back a producer: the producers are
      // dispatched ahead of it and wait on nothing.
      constexpr long SLOT = 4L * 8 * NJ * 64;  // float4 per partial tile
      float4* slot = reinterpret_cast<float4*>(p.ws) + ((long)tb * (nsplit - 1) + ks) * SLOT +
                     (long)wid * (8 * NJ * 64) + lane;
      int* flags = p.tick + (long)tb * 8;
      if (ks < nsplit - 1) {
        // stored straight from the AGPRs (asm "a" operands, no VGPR copies of the accumulators);
        // 1 KiB per wave store, 4 stores per 4 KiB window of the base (13-bit signed immediate)
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
          for (int j = 0; j < NJ; ++j)
            asm volatile("global_store_dwordx4 %0, %1, off offset:%2"
                         :
                         : "v"(slot + (long)(i * NJ + (j & ~3)) * 64), "a"(acc[i][j]), "i"((j & 3) * 1024)
                         : "memory");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (wid == 0 && !(p.dbg & 2)) {  // the whole wave (one address, one value)
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          __hip_atomic_store(flags + ks, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        probe_end();
        return;
      }
      __shared__ int lost;  // a producer's flag never came
      if (wid == 0) {
        // lane l watches slice (l & 7)'s flag; bounded (p.spin polls, a few seconds by default) so
        // a broken hand-off cannot hang the GPU
        int* fl = flags + (lane & 7);
        const bool watch = (lane & 7) < nsplit - 1;
        int v = 0;
        for (int n = 0; n < p.spin; ++n) {
          v = __hip_atomic_load(fl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          if (__all(!watch || v != 0)) break;
          __builtin_amdgcn_s_sleep(4);
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        // re-arm only the flags seen raised: one never seen may still be raised by a late producer,
        // and the error word makes that launch (and the buffer) visibly bad instead of silently
        const bool miss = watch && v == 0;
        if (!miss) __hip_atomic_store(fl, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const bool any = __any(miss);
        if (lane == 0) {
          lost = any ? 1 : 0;
          if (any) __hip_atomic_fetch_add(p.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      split_slot = slot - (long)ks * SLOT;  // slice 0's partial; the epilogue adds them as it converts
      split_lost = __builtin_amdgcn_readfirstlane(lost);
    }
  }

  // ---- epilogue through LDS: quadrant rows of 256 B (NW * 2 used), chunk c at c ^ (row & 15),
  // its two 8-B halves swapped in rows with bit 3 set (stg_swap): a fragment write is a
  // ds_write_b64 whose 16-lane groups hold rows lr = 0..15 of one column chunk; banks are
  // (a / 4) % 32 for every LDS write, so the XOR alone puts them on 8 chunk positions x 1 half
  // = 16 of the 32 banks (2-way, 4 extra cycles per write: the 1024 SQ_LDS_BANK_CONFLICT per
  // tile of round 5); the half swap gives 8 x 2 = all 32
  barrier();  // every wave is done with the stages before they become epilogue staging
  char* wl = smem + wid * 32768;
  {
    const int lr = lane & 15, hc = lane >> 4;  // acc row, 4-column group of the fragment
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int m = i * 16 + lr;
      // split-K: the partials of slices 0 .. S-2 summed in slice order, then + this slice's own
      // accumulators (fragment order, one row of fragments at a time: the sums are consumed
      // here, never all live at once)
      float4 ps[NJ];
      if (split_slot != nullptr) {
#pragma unroll
        for (int j = 0; j < NJ; ++j) ps[j] = split_slot[(i * NJ + j) * 64];
        for (int sl = 1; sl < nsplit - 1; ++sl) {
          const float4* q = split_slot + (long)sl * (4L * 8 * NJ * 64);
#pragma unroll
          for (int j = 0; j < NJ; ++j) {
            const float4 t = q[(i * NJ + j) * 64];
            ps[j].x += t.x;
            ps[j].y += t.y;
            ps[j].z += t.z;
            ps[j].w += t.w;
          }
        }
      }
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int ch = 2 * j + (hc >> 1);
        f32x4_t v = acc[i][j];
        if (split_slot != nullptr) {
          v[0] = ps[j].x + v[0];
          v[1] = ps[j].y + v[1];
          v[2] = ps[j].z + v[2];
          v[3] = ps[j].w + v[3];
          if (split_lost) v = f32x4_t{__builtin_nanf(""), __builtin_nanf(""), __builtin_nanf(""), __builtin_nanf("")};
        }
        uint2 pk;
        pk.x = pk2<E>(v[0], v[1]);
        pk.y = pk2<E>(v[2], v[3]);
        *reinterpret_cast<uint2*>(wl + m * 256 + ((ch ^ (m & 15)) << 4) + (((hc ^ (m >> 3)) & 1) << 3)) = pk;
      }
    }
  }
  __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's LDS writes landed
  __builtin_amdgcn_wave_barrier();
#ifdef FT_W4_PROBE
  pt3 = __builtin_amdgcn_s_memrealtime();
#endif
  const int cc = lane & 15;
  float sq = 0.f;  // sum of squares of the stored values (p.part)
  if constexpr (EPI == W4_SWIGLU_BWD) {
    // dgu from da (LDS) and the saved gu (global): the gu rows of 16 tile rows are loaded before
    // any is used (the fragment registers are free now), so the epilogue waits on HBM latency twice
    // per tile instead of once per 4 rows
    if (cc < 2 * NJ) {
      const int gn = n0 + wn * NW + cc * 8;
#pragma unroll
      for (int hb = 0; hb < 2; ++hb) {
        uint4 g16[16], u16[16];
#pragma unroll
        for (int q = 0; q < 16; ++q) {
          const long gm = m0 + wm * 128 + (hb * 16 + q) * 4 + (lane >> 4);
          g16[q] = *reinterpret_cast<const uint4*>(p.r + gm * p.ldr + gn);
          u16[q] = *reinterpret_cast<const uint4*>(p.r + gm * p.ldr + p.ffn + gn);
        }
#pragma unroll
        for (int q = 0; q < 16; ++q) {
          const int row = (hb * 16 + q) * 4 + (lane >> 4);
          const long gm = m0 + wm * 128 + row;
          const uint4 v = stg_swap(*reinterpret_cast<const uint4*>(wl + row * 256 + ((cc ^ (row & 15)) << 4)),
                                   (q >> 1) & 1);  // (row & 8: constant in the unrolled loop)
          // v = da (bf16, as the unfused path's GEMM output) for features gn .. gn + 7 of token gm:
          // dg, du from the saved g = gu[gm, gn], u = gu[gm, F + gn] (swiglu_grad, common.h)
          float d8[8], g8[8], u8[8], dg[8], du[8];
          unpack8e<E>(v, d8);
          unpack8e<E>(g16[q], g8);
          unpack8e<E>(u16[q], u8);
#pragma unroll
          for (int e = 0; e < 8; ++e) swiglu_grad(g8[e], u8[e], d8[e], p.exact, dg[e], du[e]);
          *reinterpret_cast<uint4*>(p.c + gm * p.ldc + gn) = pack8e<E>(dg);
          *reinterpret_cast<uint4*>(p.c + gm * p.ldc + p.ffn + gn) = pack8e<E>(du);
        }
      }
    }
  } else if (cc < 2 * NJ) {
    // the store loop in two copies: a tail tile's guards rows past M (not stored, nor summed), every
    // other tile runs without the per-row compare (mtail is uniform; only the dW layout has tails)
    auto store_rows = [&](auto tail_tag) {
      constexpr bool TAIL = decltype(tail_tag)::value;
      for (int r4 = 0; r4 < 32; r4 += 4)
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int rr = r4 + u;
        const int row = rr * 4 + (lane >> 4);
        const long gm = m0 + wm * 128 + row;
        if constexpr (TAIL) {
          if (gm >= p.M) continue;
        }
        uint4 v = stg_swap(*reinterpret_cast<const uint4*>(wl + row * 256 + ((cc ^ (row & 15)) << 4)),
                           u >> 1);  // row & 8 == (rr & 2) * 4: constant per unrolled copy
        // W4_SWIGLU: wave column half 0 holds g (gu columns [0, F)), half 1 holds u ([F, 2F))
        const int gn = EPI == W4_SWIGLU ? (wn ? p.ffn : 0) + f0 + cc * 8 : n0 + wn * NW + cc * 8;
        if constexpr (EPI == W4_RES) {
          float a[8], r[8];
          unpack8e<E>(v, a);
          unpack8e<E>(*reinterpret_cast<const uint4*>(p.r + gm * p.ldr + gn), r);
#pragma unroll
          for (int q = 0; q < 8; ++q) a[q] += r[q];
          v = pack8e<E>(a);
        } else if constexpr (EPI == W4_ROPE) {
          if (gn < p.rope_cols) {
            // 8 columns = 4 interleaved (x0, x1) pairs of one head: rotated in fp32 by the bf16
            // projection output, as the separate kernel did (rope.hip / model.py:121-126)
            const int pos = (int)(gm % p.rope_seq);
            const int i0 = (gn % p.rope_hd) >> 1;
            const float* cs = p.cos_t + (long)pos * (p.rope_hd >> 1) + i0;
            const float* sn = p.sin_t + (long)pos * (p.rope_hd >> 1) + i0;
            const float4 c4 = *reinterpret_cast<const float4*>(cs);
            const float4 s4 = *reinterpret_cast<const float4*>(sn);
            float a[8];
            unpack8e<E>(v, a);
            const float cv[4] = {c4.x, c4.y, c4.z, c4.w}, sv[4] = {s4.x, s4.y, s4.z, s4.w};
            float o[8];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              o[2 * q] = a[2 * q] * cv[q] - a[2 * q + 1] * sv[q];
              o[2 * q + 1] = a[2 * q] * sv[q] + a[2 * q + 1] * cv[q];
            }
            v = pack8e<E>(o);
          }
        }
        if (p.part != nullptr) {
          float a[8];
          unpack8e<E>(v, a);
#pragma unroll
          for (int q = 0; q < 8; ++q) sq = fmaf(a[q], a[q], sq);
        }
        if (!(p.dbg & 1)) *reinterpret_cast<uint4*>(p.c + gm * p.ldc + gn) = v;
      }
    };
    if (mtail)
      store_rows(std::true_type{});
    else
      store_rows(std::false_type{});
  }
  if (p.part != nullptr) {  // uniform: one partial per tile, fixed order (deterministic)
    sq = wave_sum(sq);
    __syncthreads();  // every wave is done with its staging quadrant
    float* red = reinterpret_cast<float*>(smem);
    if (lane == 0) red[wid] = sq;
    __syncthreads();
    if (tid == 0) p.part[tn * p.tiles_m + tm] = (red[0] + red[1]) + (red[2] + red[3]);
    // a sink's slice can hold more slots than this tile grid (sized for the smallest tile, and
    // written whole by the fallback pass): stale partials there would enter the global norm
    if (tb == 0)  // (tile 0's epilogue workgroup: with split-K its first half exits early)
      for (int i = ntiles + tid; i < p.part_n; i += NT) p.part[i] = 0.f;
  }
  if constexpr (EPI == W4_SWIGLU) {
    // a = silu(g) * u from the parked bf16 g / u quadrants (the values just stored to gu, so a is
    // bitwise what swiglu_fwd_t computes from gu): wave (wm, wn) takes rows [64 wn, 64 wn + 64) of
    // its row half, writes a row-major and back over g in LDS, then all waves store a^T
    __syncthreads();
    char* gl = smem + (wm * 2) * 32768;      // g quadrant of this row half
    char* ul = smem + (wm * 2 + 1) * 32768;  // u quadrant
    if (cc < 2 * NJ) {
      for (int r4 = 0; r4 < 16; r4 += 4)
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int row = wn * 64 + (r4 + u) * 4 + (lane >> 4);
        const int off = row * 256 + ((cc ^ (row & 15)) << 4);
        const bool sw = u >> 1;  // row & 8
        float g8[8], u8[8], a8[8];
        unpack8e<E>(stg_swap(*reinterpret_cast<const uint4*>(gl + off), sw), g8);
        unpack8e<E>(stg_swap(*reinterpret_cast<const uint4*>(ul + off), sw), u8);
#pragma unroll
        for (int q = 0; q < 8; ++q) a8[q] = g8[q] * sigmoid_f(g8[q], p.exact) * u8[q];
        const uint4 av = pack8e<E>(a8);
        *reinterpret_cast<uint4*>(p.act + (m0 + wm * 128 + row) * (long)p.ffn + f0 + cc * 8) = av;
        *reinterpret_cast<uint4*>(gl + off) = stg_swap(av, sw);
      }
    }
    if (p.actT == nullptr) {  // uniform
      probe_end();
      return;
    }
    __syncthreads();
    // a^T [F, M]: a thread takes 8 tokens x 8 features (8 row-chunk LDS reads, feature chunk
    // fastest across lanes: distinct XOR-swizzled chunks, conflict-free), transposes the block in
    // registers and stores 8 16-B pieces (8 tokens of one feature each)
    constexpr int CH = 2 * NJ;  // 8-feature chunks per tile row
    for (int k = tid; k < 2 * 16 * CH; k += NT) {
      const int fc = k % CH, tg = (k / CH) % 16, hf = k / (16 * CH);
      const char* al = smem + (hf * 2) * 32768;  // a of row half hf (written over g)
      uint16_t e[8][8];                          // [token][feature]
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int row = tg * 8 + i;
        const uint4 v = stg_swap(*reinterpret_cast<const uint4*>(al + row * 256 + ((fc ^ (row & 15)) << 4)), tg & 1);
        const uint32_t wv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          e[i][2 * q] = (uint16_t)(wv[q] & 0xffffu);
          e[i][2 * q + 1] = (uint16_t)(wv[q] >> 16);
        }
      }
      bf16_t* dst = p.actT + (long)(f0 + fc * 8) * p.M + m0 + hf * 128 + tg * 8;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        uint4 o;
        o.x = e[0][j] | ((uint32_t)e[1][j] << 16);
        o.y = e[2][j] | ((uint32_t)e[3][j] << 16);
        o.z = e[4][j] | ((uint32_t)e[5][j] << 16);
        o.w = e[6][j] | ((uint32_t)e[7][j] << 16);
        *reinterpret_cast<uint4*>(dst + (long)j * p.M) = o;
      }
    }
  }
  probe_end();
}

template <class E, int NJ, bool AT, bool BT>
void launch_nj(const W4Args& p, int epi, hipStream_t st) {
  const dim3 g(p.tiles_m * p.tiles_n * (p.splits > 1 ? p.splits : 1));
  if constexpr (!AT && !BT) {
    if (epi == W4_ROPE) {
      hipLaunchKernelGGL((gemm_w4_kernel<E, NJ, W4_ROPE, false, false>), g, dim3(NT), 0, st, p);
      return;
    }
    if (epi == W4_SWIGLU) {
      hipLaunchKernelGGL((gemm_w4_kernel<E, NJ, W4_SWIGLU, false, false>), g, dim3(NT), 0, st, p);
      return;
    }
  }
  if constexpr (!AT && BT) {
    if (epi == W4_SWIGLU_BWD) {
      hipLaunchKernelGGL((gemm_w4_kernel<E, NJ, W4_SWIGLU_BWD, false, true>), g, dim3(NT), 0, st, p);
      return;
    }
  }
  TORCH_CHECK(epi == W4_STORE || epi == W4_RES, "gemm_w4: epilogue ", epi, " not built for this layout");
  if (epi == W4_RES)
    hipLaunchKernelGGL((gemm_w4_kernel<E, NJ, W4_RES, AT, BT>), g, dim3(NT), 0, st, p);
  else
    hipLaunchKernelGGL((gemm_w4_kernel<E, NJ, W4_STORE, AT, BT>), g, dim3(NT), 0, st, p);
}

template <bool AT, bool BT>
void launch_l(at::ScalarType st_, int nj, const W4Args& p, int epi, hipStream_t st) {
  FT_DISPATCH_E16(st_, {
    switch (nj) {
      case 8: launch_nj<E, 8, AT, BT>(p, epi, st); break;
      case 7: launch_nj<E, 7, AT, BT>(p, epi, st); break;
      case 6: launch_nj<E, 6, AT, BT>(p, epi, st); break;
      default: launch_nj<E, 4, AT, BT>(p, epi, st); break;
    }
  });
}

// one translation unit per operand layout (the three compile in parallel):
//   gemm_w4_fwd.hip  K-contiguous A and B  (forward: store / residual / RoPE / SwiGLU epilogues)
//   gemm_w4_dx.hip   K-contiguous A, k-major B  (dX: store / accumulate / SwiGLU-backward)
//   gemm_w4_dw.hip   k-major A and B  (dW: store / accumulate, sums of squares)
void launch_fwd(at::ScalarType st_, int nj, const W4Args& p, int epi, hipStream_t st);
void launch_dx(at::ScalarType st_, int nj, const W4Args& p, int epi, hipStream_t st);
void launch_dw(at::ScalarType st_, int nj, const W4Args& p, int epi, hipStream_t st);

}  // namespace ftw4
