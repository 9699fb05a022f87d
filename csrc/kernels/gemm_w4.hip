// 4-wave bf16 / fp16 GEMM for gfx950 with an instruction-level schedule (the "w4" kernel).
//
//   C[M, N] = sum_k A(m, k) * B(k, n)   A = [M, K] row-major (K contiguous), B = [N, K] row-major
//   (the forward x W^T of every nn.Linear: reference model.py:195,215,254,379)
//
// Structure (one workgroup = one 256 x BN output tile, BN = 32 * NJ, BK = 64):
//   * 4 waves, one per SIMD, each owning a 128 x (16 NJ) quadrant = 8 x NJ fragments of
//     v_mfma_f32_16x16x32_bf16 (_f16 for --model-dtype fp16); the accumulators are pinned in AGPRs (the MFMAs are inline asm on
//     "+a" operands, so the compiler never shuffles them), the operand fragments in VGPRs.
//     NJ is chosen per shape so the tile count fills the 256 CUs in whole rounds (the 8B step:
//     qkv 256 x 192 -> 256 tiles, w13 256 x 224 -> 4 x 256, wo / w2 256 x 128 -> 256, head 256^2).
//   * Both operands are staged by LDS-DMA (buffer_load_dwordx4 ... lds: 1 KiB = 8 rows x 128 B per
//     wave-instruction, no staging VGPRs; the per-lane source offset XOR-swizzled so the
//     ds_read_b128 fragment reads are bank-conflict free: chunk c of row r sits at c ^ (r & 7)),
//     double-buffered (2 stages of 32 + 4 NJ KiB).
//   * One K-tile = 2 x 8 NJ MFMAs per wave (two k-steps of 32). The fragment registers are
//     double-buffered by k-step, so every LDS read is issued right behind an MFMA and consumed a
//     k-step later:
//       MFMA 0 .. R-1 : the k-step-1 fragment reads of this tile (R = 8 + NJ ds_read_b128)
//       MFMA 24       : lgkmcnt(0) + barrier  -> every wave has finished reading this stage
//       then          : the 8 + NJ LDS-DMAs of tile t+2 into this stage, spread evenly
//       MFMA SB2      : vmcnt(8 + NJ) + barrier -> tile t+1 (issued one K-tile ago) has landed
//       then          : the k-step-0 fragment reads of tile t+1
//     This is the counts-and-placement schedule of the vendor's tuned assembly GEMMs on this chip
//     (one wave per SIMD, direct-to-LDS, prefetch two tiles ahead), with HIP choosing registers.
//   * Epilogue through LDS: per-lane stores straight from the MFMA accumulator layout write 16
//     rows x 32 B per instruction and cost 20-26 % of the kernel (ablation in
//     profiles/r3_gemm_w4_investigation.md); each wave instead parks its quadrant in 32 KiB of the
//     idle LDS (256-B rows, 16-B chunks XOR-swizzled by row: conflict-free 8-B writes and 16-B
//     row reads) and stores whole rows, 4 x 256 B per instruction. Fused epilogues act on the
//     row-contiguous values: + residual (wo / w2 into the residual stream), RoPE on the packed
//     Q/K columns of the QKV projection (reference model.py:100-126: interleaved pairs, fp32).
//   * Tiles are mapped XCD-contiguously (blockIdx % 8 = XCD under round-robin dispatch),
//     M-fastest inside an XCD's range, so the XCD's L2 serves the shared B panel.
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

constexpr int BM = 256, BK = 64, NT = 256;
constexpr int PIECE = 1024;  // one LDS-DMA wave-instruction: 8 image rows of 128 B
constexpr int FS = 2 * PIECE;  // one 16-row fragment
constexpr int OPA = 32 * PIECE;  // A image: 256 rows

enum W4Epi : int { W4_STORE = 0, W4_RES = 1, W4_ROPE = 2, W4_SWIGLU = 3 };

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
// is not saved; gfx950 needs no wait state between the m0 write and the DMA.
template <int IMM>
__device__ __forceinline__ void dma16(const i32x4_t& srd, unsigned voff, unsigned soff, unsigned sbase) {
  asm volatile("s_add_u32 m0, %2, %4\n\tbuffer_load_dwordx4 %0, %1, %3 offen lds"
               :
               : "v"(voff), "s"(srd), "s"(sbase), "s"(soff), "i"(IMM)
               : "memory");
}

template <int OFF>
__device__ __forceinline__ void ds16(bf16x8_t& d, unsigned addr) {
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(d) : "v"(addr), "i"(OFF) : "memory");
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
  asm volatile("s_waitcnt lgkmcnt(%0)" ::"i"(N) : "memory");
}
template <int N>
__device__ __forceinline__ void vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"i"(N) : "memory");
}
__device__ __forceinline__ void barrier() { asm volatile("s_barrier" ::: "memory"); }

// the registers an asm wait covered: consumers stay behind the wait
__device__ __forceinline__ void tie(bf16x8_t& x) { asm volatile("" : "+v"(x)); }

struct W4Args {
  const bf16_t* a;
  const bf16_t* b;
  bf16_t* c;
  const bf16_t* r;       // residual (may alias c) or null
  const float* cos_t;    // RoPE: [S, D/2] tables
  const float* sin_t;
  long lda, ldb, ldc, ldr;
  int M, N, K;
  int tiles_m, tiles_n;
  int rope_cols;         // RoPE: columns [0, rope_cols) are rotated (Hq + Hkv heads)
  int rope_hd;           // head dim
  int rope_seq;          // sequence length (position = row % seq)
  // SwiGLU epilogue (W4_SWIGLU): b = [w1; w3] ([2F, K]); tile tn covers features
  // [tn * 16 NJ, +16 NJ) of BOTH halves (B image rows = that slice of w1, then of w3), so the
  // tile holds g and u of the same features: c = gu [M, 2F], a = silu(g) u [M, F], a^T [F, M]
  int ffn;               // F
  bf16_t* act;           // a
  bf16_t* actT;          // a^T
  int exact;             // IEEE division in the sigmoid (FT_EXACT_MATH), as swiglu_fwd_t
};

__device__ __forceinline__ void tile_of(int bid, int tiles_m, int tiles_n, int& tm, int& tn) {
  const int nwg = tiles_m * tiles_n;
  const int q = nwg / 8, rem = nwg % 8;
  const int x = bid % 8, o = bid / 8;
  const int w = (x < rem ? x * (q + 1) : rem * (q + 1) + (x - rem) * q) + o;
  tm = w % tiles_m;
  tn = w / tiles_m;
}

template <int NJ>
struct Frags {
  bf16x8_t a0[8], b0[NJ], a1[8], b1[NJ];
};

template <int NJ>
struct Sched {
  static constexpr int MH = 8 * NJ;          // MFMAs per k-step
  static constexpr int R = 8 + NJ;           // fragment reads per k-step: b[0], a[0..7], b[1..]
  static constexpr int D = 8 + NJ;           // LDS-DMAs per wave per K-tile (A 8, B NJ)
  static constexpr int SB1 = 24;             // first barrier (after MFMA 24)
  static constexpr int SB2 = 2 * MH - R - 4; // second barrier
  static constexpr int dma_slot(int d) { return SB1 + 2 + d * (SB2 - SB1 - 4) / D; }
  static constexpr int OPB = NJ * 4 * PIECE;  // B image
  static constexpr int ST = OPA + OPB;        // stage
  static_assert(R <= 16 && SB2 - SB1 - 4 >= D && SB2 + R < 2 * MH, "schedule does not fit");
};

// lane's part of read r (b[0], a[0..7], b[1..NJ-1]) into the fragment arrays
template <int NJ, int r>
__device__ __forceinline__ void rd(bf16x8_t (&ax)[8], bf16x8_t (&bx)[NJ], unsigned ab, unsigned bb) {
  if constexpr (r == 0)
    ds16<0>(bx[0], bb);
  else if constexpr (r <= 8)
    ds16<FS * (r - 1)>(ax[r - 1], ab);
  else
    ds16<FS * (r - 8)>(bx[r - 8], bb);
}

struct Ctx {
  i32x4_t srdA, srdB;
  unsigned voA[8], voB[8];
  unsigned rdA0, rdA1, rdB0, rdB1;
  unsigned lds0;
  int wid;
};

// One K-tile t (stage cur = t & 1): DMA: stage tile t + 2 into this stage; NEXT: read tile t + 1's
// first k-step.
template <class E, int NJ, bool DMA, bool NEXT>
__device__ __forceinline__ void ktile(f32x4_t (&acc)[8][NJ], Frags<NJ>& f, int t, const Ctx& c) {
  using S = Sched<NJ>;
  const unsigned cur = (unsigned)(t & 1) * S::ST, nxt = (unsigned)((t + 1) & 1) * S::ST;
  const unsigned a1b = c.rdA1 + cur, b1b = c.rdB1 + cur, a0n = c.rdA0 + nxt, b0n = c.rdB0 + nxt;
  const unsigned kofs = (unsigned)(t + 2) * (BK * 2);
  const unsigned sb = __builtin_amdgcn_readfirstlane(c.lds0 + cur + c.wid * PIECE);
  sfor<2 * S::MH>([&](auto SS) {
    constexpr int s = SS;
    constexpr int i = s & 7, j = (s % S::MH) >> 3;  // runs of 8 MFMAs share the B fragment (SrcA)
    if constexpr (s == 0) {  // the first run's 9 fragments landed (issued last K-tile)
      lgkm<S::R - 9>();
      tie(f.b0[0]);
      sfor<8>([&](auto I) { tie(f.a0[I]); });
    }
    if constexpr (s == 8) {  // all of k-step 0 (8 newer reads in flight)
      lgkm<8>();
      sfor<NJ>([&](auto J) { tie(f.b0[J]); });
    }
    if constexpr (s == 2) asm volatile("s_setprio 3" ::: "memory");
    if constexpr (s < S::MH)
      mfma<E>(acc[i][j], f.b0[j], f.a0[i]);
    else
      mfma<E>(acc[i][j], f.b1[j], f.a1[i]);
    if constexpr (s < S::R) rd<NJ, s>(f.a1, f.b1, a1b, b1b);
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
            dma16<qa * 4 * PIECE>(c.srdA, c.voA[qa], kofs, sb);
          else
            dma16<OPA + (d / 2) * 4 * PIECE>(c.srdB, c.voB[d / 2], kofs, sb);
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
    if constexpr (NEXT && s > S::SB2 && s <= S::SB2 + S::R) rd<NJ, s - S::SB2 - 1>(f.a0, f.b0, a0n, b0n);
    if constexpr (s == 2 * S::MH - 1) asm volatile("s_setprio 0" ::: "memory");
  });
}

template <class E, int NJ, int EPI>
__global__ __launch_bounds__(NT, 1) void gemm_w4_kernel(W4Args p) {
  using S = Sched<NJ>;
  constexpr int LDS = 2 * S::ST > 4 * 32768 ? 2 * S::ST : 4 * 32768;  // stages / epilogue staging
  __shared__ __attribute__((aligned(1024))) char smem[LDS];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid >> 1, wn = wid & 1;
  constexpr int BN = 32 * NJ, NW = 16 * NJ;
  int tm, tn;
  tile_of(blockIdx.x, p.tiles_m, p.tiles_n, tm, tn);
  const int m0 = tm * BM, n0 = tn * BN;
  const int f0 = tn * NW;  // W4_SWIGLU: first feature of the tile (NW features of w1 and of w3)
  const int nk = p.K / BK;

  // LDS-DMA sources: instruction q of wave w covers image rows (q * 4 + w) * 8 + (lane >> 3);
  // lane's 16-B chunk (lane & 7) holds global chunk (lane & 7) ^ (row & 7)
  Ctx c;
  c.wid = wid;
  c.srdA = make_srd(p.a + (long)m0 * p.lda);
  c.srdB = make_srd(EPI == W4_SWIGLU ? p.b : p.b + (long)n0 * p.ldb);
  const int lrow = wid * 8 + (lane >> 3), lch = (lane & 7) ^ (lane >> 3);
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    c.voA[q] = (unsigned)(((q * 32 + lrow) * p.lda + lch * 8) * 2);
    const int r = q * 32 + lrow;  // B image row
    const long src = EPI == W4_SWIGLU ? (r < 16 * NJ ? f0 + r : (long)p.ffn + f0 + (r - 16 * NJ)) : r;
    c.voB[q] = (unsigned)((src * p.ldb + lch * 8) * 2);
  }
  c.lds0 = __builtin_amdgcn_readfirstlane(lds_u32(smem));
  // fragment reads: lane reads row r0 + (lane & 15), chunk (kk * 4 + (lane >> 4)) ^ (lane & 7)
  const unsigned lrowb = (unsigned)(((lane & 15) >> 3) * PIECE + (lane & 7) * 128);
  const unsigned lpart0 = lrowb + (unsigned)((((lane >> 4)) ^ (lane & 7)) << 4);
  const unsigned lpart1 = lrowb + (unsigned)(((4 + (lane >> 4)) ^ (lane & 7)) << 4);
  c.rdA0 = c.lds0 + wm * 16 * PIECE + lpart0;
  c.rdA1 = c.lds0 + wm * 16 * PIECE + lpart1;
  c.rdB0 = c.lds0 + OPA + wn * NJ * 2 * PIECE + lpart0;
  c.rdB1 = c.lds0 + OPA + wn * NJ * 2 * PIECE + lpart1;

  f32x4_t acc[8][NJ];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  Frags<NJ> f;

  // prologue: tiles 0 and 1 in flight, then tile 0's k-step-0 fragments
  const unsigned sb0 = __builtin_amdgcn_readfirstlane(c.lds0 + wid * PIECE);
  const unsigned sb1 = __builtin_amdgcn_readfirstlane(c.lds0 + S::ST + wid * PIECE);
  sfor<8>([&](auto Q) { dma16<Q * 4 * PIECE>(c.srdA, c.voA[Q], 0u, sb0); });
  sfor<NJ>([&](auto Q) { dma16<OPA + Q * 4 * PIECE>(c.srdB, c.voB[Q], 0u, sb0); });
  if (nk > 1) {
    sfor<8>([&](auto Q) { dma16<Q * 4 * PIECE>(c.srdA, c.voA[Q], (unsigned)(BK * 2), sb1); });
    sfor<NJ>([&](auto Q) { dma16<OPA + Q * 4 * PIECE>(c.srdB, c.voB[Q], (unsigned)(BK * 2), sb1); });
    vmcnt<S::D>();
  } else {
    vmcnt<0>();
  }
  barrier();
  sfor<S::R>([&](auto RR) { rd<NJ, RR>(f.a0, f.b0, c.rdA0, c.rdB0); });

  // the zeroed accumulators are MFMA sources next (VALU write -> MFMA SrcC wait states)
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_nop 4" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
  int t = 0;
  for (; t + 2 < nk; ++t) ktile<E, NJ, true, true>(acc, f, t, c);
  if (nk >= 2) {
    ktile<E, NJ, false, true>(acc, f, t, c);
    ++t;
  }
  ktile<E, NJ, false, false>(acc, f, t, c);
  // The accumulators are read by VALU next: wait out the last MFMAs (the compiler does not see
  // the asm as MFMAs, so it inserts no wait states), and keep every accumulator read behind the
  // pad (sched_barrier: register-only instructions may otherwise be hoisted above an asm).
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);

  // ---- epilogue through LDS: quadrant rows of 256 B (NW * 2 used), chunk c at c ^ (row & 15)
  barrier();  // every wave's last fragment reads are done (no DMA is in flight)
  char* wl = smem + wid * 32768;
  {
    const int lr = lane & 15, hc = lane >> 4;  // acc row, 4-column group of the fragment
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int m = i * 16 + lr;
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int ch = 2 * j + (hc >> 1);
        const f32x4_t v = acc[i][j];
        uint2 o;
        o.x = pk2<E>(v[0], v[1]);
        o.y = pk2<E>(v[2], v[3]);
        *reinterpret_cast<uint2*>(wl + m * 256 + ((ch ^ (m & 15)) << 4) + (hc & 1) * 8) = o;
      }
    }
  }
  __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's LDS writes landed
  __builtin_amdgcn_wave_barrier();
  const int cc = lane & 15;
  if (cc < 2 * NJ) {
#pragma unroll 4
    for (int rr = 0; rr < 32; ++rr) {
      const int row = rr * 4 + (lane >> 4);
      uint4 v = *reinterpret_cast<const uint4*>(wl + row * 256 + ((cc ^ (row & 15)) << 4));
      const long gm = m0 + wm * 128 + row;
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
      *reinterpret_cast<uint4*>(p.c + gm * p.ldc + gn) = v;
    }
  }
  if constexpr (EPI == W4_SWIGLU) {
    // a = silu(g) * u from the parked bf16 g / u quadrants (the values just stored to gu, so a is
    // bitwise what swiglu_fwd_t computes from gu): wave (wm, wn) takes rows [64 wn, 64 wn + 64) of
    // its row half, writes a row-major and back over g in LDS, then all waves store a^T
    __syncthreads();
    char* gl = smem + (wm * 2) * 32768;      // g quadrant of this row half
    char* ul = smem + (wm * 2 + 1) * 32768;  // u quadrant
    if (cc < 2 * NJ) {
#pragma unroll 4
      for (int rr = 0; rr < 16; ++rr) {
        const int row = wn * 64 + rr * 4 + (lane >> 4);
        const int off = row * 256 + ((cc ^ (row & 15)) << 4);
        float g8[8], u8[8], a8[8];
        unpack8e<E>(*reinterpret_cast<const uint4*>(gl + off), g8);
        unpack8e<E>(*reinterpret_cast<const uint4*>(ul + off), u8);
#pragma unroll
        for (int q = 0; q < 8; ++q) a8[q] = g8[q] * sigmoid_f(g8[q], p.exact) * u8[q];
        const uint4 av = pack8e<E>(a8);
        *reinterpret_cast<uint4*>(p.act + (m0 + wm * 128 + row) * (long)p.ffn + f0 + cc * 8) = av;
        *reinterpret_cast<uint4*>(gl + off) = av;
      }
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
        const uint4 v = *reinterpret_cast<const uint4*>(al + row * 256 + ((fc ^ (row & 15)) << 4));
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
}

template <class E, int NJ>
void launch_nj(const W4Args& p, int epi, hipStream_t st) {
  const dim3 g(p.tiles_m * p.tiles_n);
  if (epi == W4_RES)
    hipLaunchKernelGGL((gemm_w4_kernel<E, NJ, W4_RES>), g, dim3(NT), 0, st, p);
  else if (epi == W4_ROPE)
    hipLaunchKernelGGL((gemm_w4_kernel<E, NJ, W4_ROPE>), g, dim3(NT), 0, st, p);
  else if (epi == W4_SWIGLU)
    hipLaunchKernelGGL((gemm_w4_kernel<E, NJ, W4_SWIGLU>), g, dim3(NT), 0, st, p);
  else
    hipLaunchKernelGGL((gemm_w4_kernel<E, NJ, W4_STORE>), g, dim3(NT), 0, st, p);
}

void launch(at::ScalarType st_, int nj, const W4Args& p, int epi, hipStream_t st) {
  FT_DISPATCH_E16(st_, {
    switch (nj) {
      case 8: launch_nj<E, 8>(p, epi, st); break;
      case 7: launch_nj<E, 7>(p, epi, st); break;
      case 6: launch_nj<E, 6>(p, epi, st); break;
      default: launch_nj<E, 4>(p, epi, st); break;
    }
  });
}

// Tile width for N: whole rounds of 256 tiles where possible (M = 2048 -> 8 row tiles).
int pick_nj(long M, long N) {
  const long tm = M / BM;
  int best = 0;
  double best_cost = 1e30;
  for (int nj : {8, 7, 6, 4}) {
    const long bn = 32L * nj;
    if (N % bn) continue;
    const long tiles = tm * (N / bn);
    const long rounds = (tiles + 255) / 256;
    // time ~ rounds x tile work; a narrower tile re-reads A more per MFMA (x ~1.06 for 4)
    const double eff = nj == 8 ? 1.0 : nj == 7 ? 0.99 : nj == 6 ? 0.98 : 0.92;
    const double cost = (double)rounds * nj / eff;
    if (cost < best_cost - 1e-9) {
      best_cost = cost;
      best = nj;
    }
  }
  return best;
}

}  // namespace

// C = A @ B^T (+ residual / RoPE): A [M, K], B [N, K] bf16 row-major; M % 256, K % 64,
// N % (32 * nj) for a tile width in {256, 224, 192, 128}. nj = 0 picks the width per shape.
at::Tensor gemm_nt_w4(const at::Tensor& a, const at::Tensor& b, const std::optional<at::Tensor>& out,
                      const std::optional<at::Tensor>& residual, int64_t nj) {
  FT_CHECK_CUDA(a);
  TORCH_CHECK(a.scalar_type() == at::kBFloat16 || a.scalar_type() == at::kHalf, "gemm_nt_w4: bf16 / fp16");
  TORCH_CHECK(b.scalar_type() == a.scalar_type(), "gemm_nt_w4: A / B dtype mismatch");
  FT_CHECK_CONTIG(a);
  FT_CHECK_CONTIG(b);
  TORCH_CHECK(a.dim() == 2 && b.dim() == 2 && a.size(1) == b.size(1), "gemm_nt_w4: A [M, K], B [N, K]");
  const long M = a.size(0), K = a.size(1), N = b.size(0);
  const int NJ = nj > 0 ? (int)nj : pick_nj(M, N);
  TORCH_CHECK(NJ == 8 || NJ == 7 || NJ == 6 || NJ == 4, "gemm_nt_w4: tile width 32 * {8, 7, 6, 4}");
  TORCH_CHECK(M % BM == 0 && N % (32 * NJ) == 0 && K % BK == 0 && K >= BK, "gemm_nt_w4: M % 256, N % ",
              32 * NJ, ", K % 64 (got ", M, " ", N, " ", K, ")");
  TORCH_CHECK(M * K * 2 < (1L << 32) && N * K * 2 < (1L << 32), "gemm_nt_w4: operand over 4 GiB");
  const at::DeviceGuard guard(a.device());
  at::Tensor c;
  if (out.has_value() && out->defined()) {
    c = *out;
    TORCH_CHECK(c.scalar_type() == a.scalar_type(), "gemm_nt_w4: out dtype");
    FT_CHECK_CONTIG(c);
    TORCH_CHECK(c.numel() == M * N, "gemm_nt_w4: out has the wrong size");
  } else {
    c = at::empty({M, N}, a.options());
  }
  W4Args p{};
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
  p.tiles_n = N / (32 * NJ);
  int epi = W4_STORE;
  if (residual.has_value() && residual->defined()) {
    TORCH_CHECK(residual->scalar_type() == a.scalar_type(), "gemm_nt_w4: residual dtype");
    FT_CHECK_CONTIG((*residual));
    TORCH_CHECK(residual->numel() == M * N, "gemm_nt_w4: residual has the wrong size");
    p.r = cptr<bf16_t>(*residual);
    epi = W4_RES;
  }
  launch(a.scalar_type(), NJ, p, epi, ft_stream());
  FT_LAUNCH_CHECK();
  return c;
}

// Fused QKV projection + RoPE: qkv = x @ w^T with the first (hq + hkv) * d columns (Q and K heads)
// rotated in the epilogue (interleaved pairs, cos/sin [S, d/2] fp32 tables; row = b * S + s).
at::Tensor gemm_qkv_rope_w4(const at::Tensor& x, const at::Tensor& w, const at::Tensor& cos_t,
                            const at::Tensor& sin_t, int64_t seq, int64_t hq, int64_t hkv, int64_t d) {
  FT_CHECK_CUDA(x);
  TORCH_CHECK(x.scalar_type() == at::kBFloat16 || x.scalar_type() == at::kHalf, "gemm_qkv_rope_w4: bf16 / fp16");
  TORCH_CHECK(w.scalar_type() == x.scalar_type(), "gemm_qkv_rope_w4: x / w dtype mismatch");
  FT_CHECK_CONTIG(x);
  FT_CHECK_CONTIG(w);
  FT_CHECK_F32(cos_t);
  FT_CHECK_F32(sin_t);
  FT_CHECK_CONTIG(cos_t);
  FT_CHECK_CONTIG(sin_t);
  const long M = x.size(0), K = x.size(1), N = w.size(0);
  TORCH_CHECK(w.size(1) == K && N == (hq + 2 * hkv) * d, "gemm_qkv_rope_w4: shape mismatch");
  TORCH_CHECK(d % 8 == 0 && M % seq == 0 && cos_t.size(0) >= seq && cos_t.size(1) == d / 2,
              "gemm_qkv_rope_w4: rope tables / head dim");
  const int NJ = pick_nj(M, N);
  TORCH_CHECK(NJ > 0 && M % BM == 0 && K % BK == 0, "gemm_qkv_rope_w4: M % 256, K % 64, N % 128");
  const at::DeviceGuard guard(x.device());
  auto c = at::empty({M, N}, x.options());
  W4Args p{};
  p.a = cptr<bf16_t>(x);
  p.b = cptr<bf16_t>(w);
  p.c = mptr<bf16_t>(c);
  p.cos_t = cptr<float>(cos_t);
  p.sin_t = cptr<float>(sin_t);
  p.lda = K;
  p.ldb = K;
  p.ldc = N;
  p.M = M;
  p.N = N;
  p.K = K;
  p.tiles_m = M / BM;
  p.tiles_n = N / (32 * NJ);
  p.rope_cols = (int)((hq + hkv) * d);
  p.rope_hd = (int)d;
  p.rope_seq = (int)seq;
  launch(x.scalar_type(), NJ, p, W4_ROPE, ft_stream());
  FT_LAUNCH_CHECK();
  return c;
}

// Fused w1|w3 projection + SwiGLU (reference model.py:254 silu(w1 x) * w3 x): x [M, K],
// w13 = [w1; w3] [2F, K] -> (gu [M, 2F] = x w13^T for the backward, a = silu(g) u [M, F],
// a^T [F, M] for the w2 weight gradient). 224-column tiles: 112 features of w1 and the same 112 of
// w3; M % 256, F % 112, K % 64.
std::tuple<at::Tensor, at::Tensor, at::Tensor> gemm_swiglu_w4(const at::Tensor& x, const at::Tensor& w13) {
  FT_CHECK_CUDA(x);
  TORCH_CHECK(x.scalar_type() == at::kBFloat16 || x.scalar_type() == at::kHalf, "gemm_swiglu_w4: bf16 / fp16");
  TORCH_CHECK(w13.scalar_type() == x.scalar_type(), "gemm_swiglu_w4: x / w13 dtype mismatch");
  FT_CHECK_CONTIG(x);
  FT_CHECK_CONTIG(w13);
  const long M = x.size(0), K = x.size(1), F2 = w13.size(0), F = F2 / 2;
  constexpr int NJ = 7, NWC = 16 * NJ;
  TORCH_CHECK(w13.size(1) == K && F2 % 2 == 0, "gemm_swiglu_w4: shape mismatch");
  TORCH_CHECK(M % BM == 0 && F % NWC == 0 && K % BK == 0 && K >= BK, "gemm_swiglu_w4: M % 256, F % 112, K % 64 (got ",
              M, " ", F, " ", K, ")");
  TORCH_CHECK(M * K * 2 < (1L << 32) && F2 * K * 2 < (1L << 32), "gemm_swiglu_w4: operand over 4 GiB");
  const at::DeviceGuard guard(x.device());
  auto gu = at::empty({M, F2}, x.options());
  auto a = at::empty({M, F}, x.options());
  auto aT = at::empty({F, M}, x.options());
  W4Args p{};
  p.a = cptr<bf16_t>(x);
  p.b = cptr<bf16_t>(w13);
  p.c = mptr<bf16_t>(gu);
  p.lda = K;
  p.ldb = K;
  p.ldc = F2;
  p.M = M;
  p.N = F2;
  p.K = K;
  p.tiles_m = M / BM;
  p.tiles_n = F / NWC;
  p.ffn = (int)F;
  p.act = mptr<bf16_t>(a);
  p.actT = mptr<bf16_t>(aT);
  p.exact = (int)ft_exact_math();
  launch(x.scalar_type(), NJ, p, W4_SWIGLU, ft_stream());
  FT_LAUNCH_CHECK();
  return {gu, a, aT};
}

int64_t gemm_w4_pick(int64_t M, int64_t N) { return pick_nj(M, N); }

TORCH_LIBRARY_FRAGMENT(ftamd, m) {
  m.def("gemm_nt_w4(Tensor a, Tensor b, Tensor(a!)? out=None, Tensor? residual=None, int nj=0) -> Tensor",
        &gemm_nt_w4);
  m.def("gemm_qkv_rope_w4(Tensor x, Tensor w, Tensor cos, Tensor sin, int seq, int hq, int hkv, int d) -> Tensor",
        &gemm_qkv_rope_w4);
  m.def("gemm_w4_pick(int M, int N) -> int", &gemm_w4_pick);
  m.def("gemm_swiglu_w4(Tensor x, Tensor w13) -> (Tensor, Tensor, Tensor)", &gemm_swiglu_w4);
}
