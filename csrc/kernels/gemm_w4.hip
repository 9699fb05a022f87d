// Host API of the w4 GEMM (kernel: gemm_w4.h; instantiations: gemm_w4_{fwd,dx,dw}.hip).
#include "gemm_w4.h"

#include <map>
#include <mutex>

namespace {

using namespace ftw4;

long long* g_prof = nullptr;  // per-workgroup stamps (gemm_w4_set_prof): W4Args::prof of every launch
long g_prof_rows = 0;         // rows of that buffer (checked against the grid at launch)

extern int g_deadzero;

void launch(at::ScalarType st_, int nj, const W4Args& p_, int epi, hipStream_t st, bool at_ = false,
            bool bt = false) {
  W4Args p = p_;
  p.deadzero = g_deadzero;
  TORCH_CHECK(p.prof == nullptr || (long)p.tiles_m * p.tiles_n * (p.splits > 1 ? p.splits : 1) <= g_prof_rows,
              "gemm_w4_set_prof: the buffer needs one row of 8 int64 per workgroup");
  // the step's layouts: forward (K-contiguous both), dX (k-major B), dW (k-major both)
  TORCH_CHECK(!at_ || bt, "gemm_w4: k-major A needs a k-major B (the dW layout)");
  if (at_)
    launch_dw(st_, nj, p, epi, st);
  else if (bt)
    launch_dx(st_, nj, p, epi, st);
  else
    launch_fwd(st_, nj, p, epi, st);
}

// Tile width for N: whole rounds of 256 tiles where possible (M = 2048 -> 8 row tiles).
// kmajor_a (the dW layout, both operands k-major): the 256 x 128 tile is LDS-bound there (16
// transposed fragment reads per k-step for 32 MFMAs): measured 0.65 of the wide tile's rate per
// unit of work (8B qkv dW 6144 x 4096 x 2048: 116.4 us at 128 columns in 3 rounds vs 99.9 us at
// 256 in 2, profiles/r4_w4_dw_nj_probe.log).
int pick_nj(long M, long N, bool kmajor_a = false) {
  const long tm = (M + BM - 1) / BM;
  int best = 0;
  double best_cost = 1e30;
  for (int nj : {8, 7, 6, 4}) {
    const long bn = 32L * nj;
    if (N % bn) continue;
    const long tiles = tm * (N / bn);
    const long rounds = (tiles + 255) / 256;
    // time ~ rounds x tile work; a narrower tile re-reads A more per MFMA (x ~1.06 for 4)
    const double eff = nj == 8 ? 1.0 : nj == 7 ? 0.99 : nj == 6 ? 0.98 : (kmajor_a ? 0.65 : 0.92);
    const double cost = (double)rounds * nj / eff;
    if (cost < best_cost - 1e-9) {
      best_cost = cost;
      best = nj;
    }
  }
  return best;
}

// Split-K (gemm_w4.h, W4Args::splits): a tile grid that fills under half the chip runs each tile
// as S = 2 / 4 / 8 workgroups over slices of K of >= 16 K-tiles each (the 8B dX products with N_out
// = 4096 at M = 2048: 128 tiles of 256 columns x 2; the GPT-2 LM-head dX, N_out = 768 / 1024, K =
// V: 24 / 32 tiles x 8). FT_W4_SPLITK=0 disables it (A/B), =2 forces a split of 2 where it fits.
int g_splitk_mode = [] {
  const char* e = std::getenv("FT_W4_SPLITK");
  return e == nullptr ? 1 : std::atoi(e);
}();

struct Plan {
  int nj, splits;
};

// Per-shape tile width and split: minimise rounds of 256 workgroups x per-workgroup work, with the
// tile widths' relative main-loop rates (eff) and a fixed epilogue / split hand-off cost per tile in
// K-tile units (the split's first half writes 4 B per output element, the second reads them).
// The dW layout (k-major A) splits only its 128-wide tile (gemm_w4.h: the wider k-major tiles keep
// no registers for the hand-off): the GPT-2-sized weight gradients, 18-96 tiles at 2048 tokens.
Plan pick_plan(long M, long N, long K, bool kmajor_a, bool kmajor_b) {
  const long tm = (M + BM - 1) / BM, nkt = K / BK;
  Plan best{pick_nj(M, N, kmajor_a), 1};
  if (g_splitk_mode == 0 || best.nj == 0) return best;
  // per slice: its K-tiles, the epilogue (~3 K-tiles) and ~6 K-tiles per slice for the hand-off
  // (the partial's fp32 store, the flag, the last slice's reads): fitted to the GPT-2 products,
  // t(S) ~ a + b K/S + c S with c / b ~ 6 K-tiles (profiles/r6/gpt2_gemm_probe_*.log: the
  // GPT-2-small w1|w3 dX at S = 1 / 2 / 3 / 4: 49.7 / 35.0 / 31.9 / 32.9 us)
  // (the 8B dX / w2 products, >= 128 tiles, keep the round-5 constant of 3: their plans were
  // measured there, profiles/r5_w4_split_bench.log)
  auto cost = [&](int nj, int sp) {
    const long tiles = tm * (N / (32L * nj));
    const long rounds = (tiles * sp + 255) / 256;
    const double eff = nj == 8 ? 1.0 : nj == 7 ? 0.99 : nj == 6 ? 0.98 : (kmajor_a ? 0.65 : kmajor_b ? 0.85 : 0.92);
    const double hand = tm * (N / 256) >= 128 ? 3.0 : 6.0;
    return (double)rounds * nj * ((double)nkt / sp + 3.0 + (sp > 1 ? hand * sp : 0.0)) / eff;
  };
  double bc = cost(best.nj, 1);
  for (int nj : {8, 7, 6, 4}) {
    if (N % (32L * nj) || (kmajor_a && nj != 4)) continue;
    const long tiles = tm * (N / (32L * nj));
    // slices of >= 16 K-tiles; >= 8 for grids under half the chip with K >= 2048 (GPT-2 sizes:
    // there the split's hand-off is cheaper than idle CUs, profiles/r5_gpt2_gemm_probe2.log; the
    // 1024-deep ones gain nothing from a split)
    const long min_kt = (tiles < 128 && nkt >= 32) ? 8 : 16;
    for (int sp : {2, 3, 4, 8}) {
      if (nkt / sp < min_kt || (K / (2 * BK)) < sp) continue;
      if (tiles * sp > 256) continue;  // one round: every slice co-resident with its tile's others
      if (g_splitk_mode == 2 && sp != 2) continue;
      const double c = cost(nj, sp);
      if (c < bc - 1e-9 || (g_splitk_mode == 2 && best.splits == 1)) {
        bc = c;
        best = Plan{nj, sp};
      }
    }
  }
  return best;
}

// Split-K hand-off flags: one zeroed int32 buffer per (device, stream), grown on demand and kept
// (each tile's last slice re-arms its flags, so the buffer is zero between launches; launches on
// one stream are ordered, two streams never share flags). The buffer's last word counts hand-offs
// that timed out (W4Args::err, gemm_w4_splitk_errors). Nothing can be allocated under stream
// capture: a graph's capture stream gets its own buffer beforehand (gemm_w4_prepare_capture, from
// GraphedStep.prime), so its replays never share flags with eager launches on any stream. Without
// one the product runs unsplit (and says so once): a graph would then sum in another order than
// the eager step.
std::mutex g_tick_mu;
std::map<std::pair<int, hipStream_t>, at::Tensor> g_tick_bufs;
constexpr long TICKS = 65536;  // >= 8 x the tiles of any split plan (<= 256 workgroups) + the error word

at::Tensor& tick_buffer_locked(const c10::Device& dev, hipStream_t st) {
  auto it = g_tick_bufs.find({dev.index(), st});
  if (it != g_tick_bufs.end()) return it->second;
  static std::vector<at::Tensor> keep;  // never freed: a captured graph holds its pointer
  at::Tensor b = at::zeros({TICKS}, at::TensorOptions().device(dev).dtype(at::kInt));
  keep.push_back(b);
  return g_tick_bufs[{dev.index(), st}] = b;
}

int* splitk_ticks(const c10::Device& dev, hipStream_t st, long n) {
  std::lock_guard<std::mutex> lock(g_tick_mu);
  TORCH_CHECK(n < TICKS, "gemm_w4: split-K flag buffer too small for ", n, " flags");
  auto it = g_tick_bufs.find({dev.index(), st});
  if (it != g_tick_bufs.end()) return it->second.data_ptr<int>();
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(st, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) {
    TORCH_WARN_ONCE("gemm_w4: split-K product captured on a stream without a prepared flag buffer "
                    "(gemm_w4_prepare_capture): it runs unsplit inside the graph");
    return nullptr;
  }
  return tick_buffer_locked(dev, st).data_ptr<int>();
}

// Sets p.splits (1 or 2) and the split's hand-off words / fp32 workspace; `ws_hold` keeps the
// workspace alive until the launch is enqueued (the caching allocator orders its reuse on the
// stream). Falls back to one workgroup per tile where the split cannot run.
int g_dbg = 0;  // timing probes (gemm_w4_set_dbg): W4Args::dbg of every launch
int g_spin = 1 << 22;  // split-K consumer poll bound (gemm_w4_set_spin: tests of the timeout path)
// The last two K-tiles' DMAs (no tile t + 2 to fetch) through null descriptors instead of
// re-staging the last tile (gemm_w4_set_deadzero, FT_W4_DEADZERO: A/B)
// Round-remainder split of a 1.5-round dW grid (gemm_w4_ex; gemm_w4_set_remainder, FT_W4_REMAINDER: A/B)
int g_remainder = [] {
  const char* e = std::getenv("FT_W4_REMAINDER");
  return e == nullptr ? 1 : std::atoi(e);
}();
int g_deadzero = [] {
  const char* e = std::getenv("FT_W4_DEADZERO");
  return e == nullptr ? 1 : std::atoi(e);
}();
// Grouped tile raster (W4Args::group, tile_of): the XCD's 32 concurrent tiles as a G x 32/G block.
// -1 (default): 8 for the dW layout (k-major A), 4 or 8 per entry otherwise; >= 0 forces (0: plain).
// Measured per 8B product (scripts/w4_raster_bench.py, profiles/r5_w4_raster_sweep2.log): w13 dW
// 392 -> 348 us, head dW 1823 -> 1682, head dX 1498 -> 1442, w2 / w13 forward 1.02x; the small
// one-round products unchanged.
int g_group = -1;
// The forward NT entry (w2 / LM-head forward) and the SwiGLU-backward dX take 8 too (head forward
// 1565 -> 1533 us, SwiGLU backward 224 -> 219 us; the other products tie,
// profiles/r5_w4_raster_sweep3.log); the plain dX and the fused QKV / SwiGLU forwards take 4.
int raster_group(bool a_t, int dflt = 4) { return g_group >= 0 ? g_group : (a_t ? 8 : dflt); }

void setup_split(W4Args& p, int splits, int nj, const at::Tensor& like, at::Tensor& ws_hold, bool a_t = false) {
  p.dbg = g_dbg;
  p.prof = g_prof;
  p.splits = 1;
  if (splits < 2) return;
  TORCH_CHECK(splits <= 8, "gemm_w4: split-K of 2 .. 8");
  TORCH_CHECK(p.K / (2 * BK) >= splits, "gemm_w4: split-K needs K / 128 >= splits");
  TORCH_CHECK(!a_t || nj == 4, "gemm_w4: split-K of the dW layout (k-major A) is built for the 128-wide tile");
  const long tiles = (long)p.tiles_m * p.tiles_n;
  int* t = splitk_ticks(like.device(), ft_stream(), 8 * tiles);
  if (t == nullptr) return;
  ws_hold = at::empty({tiles * (splits - 1) * BM * 32L * nj}, like.options().dtype(at::kFloat));
  p.splits = splits;
  p.tick = t;
  p.err = t + (TICKS - 1);
  p.spin = g_spin;
  p.ws = ws_hold.data_ptr<float>();
}

}  // namespace

// C = A @ B^T (+ residual): A [M, K], B [N, K] bf16 row-major; M % 256, K % 128,
// N % (32 * nj) for a tile width in {256, 224, 192, 128}. nj = 0 picks the width per shape.
at::Tensor gemm_nt_w4(const at::Tensor& a, const at::Tensor& b, const std::optional<at::Tensor>& out,
                      const std::optional<at::Tensor>& residual, int64_t nj, int64_t splits) {
  FT_CHECK_CUDA(a);
  TORCH_CHECK(a.scalar_type() == at::kBFloat16 || a.scalar_type() == at::kHalf, "gemm_nt_w4: bf16 / fp16");
  TORCH_CHECK(b.scalar_type() == a.scalar_type(), "gemm_nt_w4: A / B dtype mismatch");
  FT_CHECK_CONTIG(a);
  FT_CHECK_CONTIG(b);
  TORCH_CHECK(a.dim() == 2 && b.dim() == 2 && a.size(1) == b.size(1), "gemm_nt_w4: A [M, K], B [N, K]");
  const long M = a.size(0), K = a.size(1), N = b.size(0);
  const Plan pl = nj > 0 ? Plan{(int)nj, (int)std::max<int64_t>(splits, 1)} : pick_plan(M, N, K, false, false);
  const int NJ = pl.nj;
  TORCH_CHECK(NJ == 8 || NJ == 7 || NJ == 6 || NJ == 4, "gemm_nt_w4: tile width 32 * {8, 7, 6, 4}");
  TORCH_CHECK(M % BM == 0 && N % (32 * NJ) == 0 && K % (2 * BK) == 0 && K > 0, "gemm_nt_w4: M % 256, N % ",
              32 * NJ, ", K % 128 (got ", M, " ", N, " ", K, ")");
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
  p.prof = g_prof;
  p.group = raster_group(false, 8);
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
  at::Tensor ws;
  setup_split(p, pl.splits, NJ, a, ws);
  launch(a.scalar_type(), NJ, p, epi, ft_stream());
  FT_LAUNCH_CHECK();
  return c;
}

// General layouts on the w4 kernel: C[M, N] (=, +=) op(A) op(B), every operand read as stored.
//   a_t = false: A is [M, K] (lda = K);  a_t = true: A is given as A^T, stored [K, M] (lda = M)
//   b_t = false: B is [N, K] (ldb = K);  b_t = true: B is stored [K, N] (ldb = N)
// dX = dY W: gemm_w4_ex(dY [T, N], false, W [N, K], true, T, K, N)
// dW = dY^T X: gemm_w4_ex(dY [T, N], true, X [T, K], true, N, K, T) (into the flat gradient
// buffer, accumulate for gradient accumulation, part: the per-tile sums of squares for the
// gradient norm, tiles_m * tiles_n floats written at part[tn * tiles_m + tm]).
at::Tensor gemm_w4_ex(const at::Tensor& a, bool a_t, const at::Tensor& b, bool b_t, int64_t M, int64_t N,
                      int64_t K, const std::optional<at::Tensor>& out, bool accumulate,
                      const std::optional<at::Tensor>& part, int64_t nj, int64_t splits) {
  FT_CHECK_CUDA(a);
  TORCH_CHECK(a.scalar_type() == at::kBFloat16 || a.scalar_type() == at::kHalf, "gemm_w4_ex: bf16 / fp16");
  TORCH_CHECK(b.scalar_type() == a.scalar_type(), "gemm_w4_ex: A / B dtype mismatch");
  FT_CHECK_CONTIG(a);
  FT_CHECK_CONTIG(b);
  TORCH_CHECK(a.numel() == M * K && b.numel() == N * K, "gemm_w4_ex: operand sizes do not match M, N, K");
  const Plan pl = nj > 0 ? Plan{(int)nj, (int)std::max<int64_t>(splits, 1)} : pick_plan(M, N, K, a_t, b_t);
  const int NJ = pl.nj;
  TORCH_CHECK(NJ == 8 || NJ == 7 || NJ == 6 || NJ == 4, "gemm_w4_ex: no tile width fits N = ", N);
  // M % 256 != 0 runs a tail tile (its rows past M clamped on load, not stored): the GPT-2 LM-head
  // dW at V = 50304 (k-major A reads 8-row chunks: M % 8)
  TORCH_CHECK((a_t ? M % 8 : M % BM) == 0 && M > 0 && N % (32 * NJ) == 0 && K % (2 * BK) == 0 && K > 0,
              "gemm_w4_ex: M % ", a_t ? 8 : BM, ", N % ", 32 * NJ, ", K % 128 (got ", M, " ", N, " ", K, ")");
  // 32-bit buffer offsets: the whole operand (a K-tile advance is a scalar offset) under 4 GiB
  TORCH_CHECK(M * K * 2 < (1L << 32) && N * K * 2 < (1L << 32), "gemm_w4_ex: operand over 4 GiB");
  const at::DeviceGuard guard(a.device());
  at::Tensor c;
  if (out.has_value() && out->defined()) {
    c = *out;
    TORCH_CHECK(c.scalar_type() == a.scalar_type(), "gemm_w4_ex: out dtype");
    FT_CHECK_CONTIG(c);
    TORCH_CHECK(c.numel() == M * N, "gemm_w4_ex: out has the wrong size");
  } else {
    TORCH_CHECK(!accumulate, "gemm_w4_ex: accumulate needs out");
    c = at::empty({M, N}, a.options());
  }
  float* part_p = nullptr;
  int part_n = 0;
  if (part.has_value() && part->defined()) {
    FT_CHECK_F32((*part));
    FT_CHECK_CONTIG((*part));
    const long need = ((M + BM - 1) / BM) * (N / (32 * NJ));
    TORCH_CHECK(part->numel() >= need, "gemm_w4_ex: part holds ", part->numel(), " partials, need ", need);
    part_p = mptr<float>(*part);
    part_n = (int)part->numel();
  }
  // rows [m_off, m_off + Ms) at tile width nj_: C rows and (k-major A) A columns offset, partials
  // from part_p + p_off (part[tn * tiles_m + tm] of this launch's grid)
  auto run = [&](long m_off, long Ms, int nj_, int splits_, long p_off) {
    W4Args p{};
    p.prof = g_prof;
    p.a = cptr<bf16_t>(a) + (a_t ? m_off : m_off * K);
    p.b = cptr<bf16_t>(b);
    p.c = mptr<bf16_t>(c) + m_off * N;
    p.r = accumulate ? p.c : nullptr;
    p.lda = a_t ? M : K;
    p.ldb = b_t ? N : K;
    p.ldc = N;
    p.ldr = N;
    p.M = Ms;
    p.N = N;
    p.K = K;
    p.tiles_m = (Ms + BM - 1) / BM;
    p.tiles_n = N / (32 * nj_);
    p.nfast = Ms > N;  // keep the larger operand's panels inside one XCD
    p.group = raster_group(a_t);
    if (part_p != nullptr) {
      p.part = part_p + p_off;
      p.part_n = part_n - (int)p_off;
    }
    at::Tensor ws;
    setup_split(p, splits_, nj_, a, ws, a_t);
    launch(a.scalar_type(), nj_, p, accumulate ? W4_RES : W4_STORE, ft_stream(), a_t, b_t);
    FT_LAUNCH_CHECK();
  };
  // Round remainder (automatic plan, dW layout): one full round of 256-wide tiles plus at most half
  // a round (the 8B qkv dW: 24 x 16 tiles = 1.5 rounds, its last round half idle) runs as two
  // launches over disjoint rows -- the full round at 256 columns, the remaining row tiles at the
  // 128-wide tile (twice as many tiles of half the work: one more full round). Same per-element
  // summation order, so bitwise the single launch's result (gemm_w4_set_remainder: A/B).
  if (nj <= 0 && a_t && g_remainder && pl.splits == 1 && NJ == 8 && N % 128 == 0 && M % BM == 0) {
    const long tn = N / 256, tm = M / BM;
    if (256 % tn == 0) {
      const long full = 256 / tn;  // row tiles of one round
      if (tm > full && (tm - full) * tn * 2 <= 256) {
        run(0, full * BM, 8, 1, 0);
        run(full * BM, M - full * BM, 4, 1, 256);
        return c;
      }
    }
  }
  run(0, M, NJ, pl.splits, 0);
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
  TORCH_CHECK(NJ > 0 && M % BM == 0 && K % (2 * BK) == 0, "gemm_qkv_rope_w4: M % 256, K % 128, N % 128");
  const at::DeviceGuard guard(x.device());
  auto c = at::empty({M, N}, x.options());
  W4Args p{};
  p.prof = g_prof;
  p.group = raster_group(false);
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
  p.splits = 1;
  launch(x.scalar_type(), NJ, p, W4_ROPE, ft_stream());
  FT_LAUNCH_CHECK();
  return c;
}

// SwiGLU tile width: 32 NJ columns = 16 NJ features of w1 and the same of w3; whole rounds of 256
// tiles at the fewest columns per CU (the 8B F = 14336: NJ 7, 4 x 256 tiles; GPT-2-small F = 2048:
// NJ 4, one round of 256; GPT-2-medium F = 2816: NJ 8, 176 tiles). 0: F fits no width.
int pick_swiglu_nj(long M, long F) {
  int best = 0;
  double best_cost = 1e30;
  for (int nj : {7, 8, 6, 4}) {
    if (F % (16L * nj)) continue;
    const long tiles = (M / BM) * (F / (16L * nj));
    const double eff = nj == 8 ? 1.0 : nj == 7 ? 0.99 : nj == 6 ? 0.98 : 0.92;
    const double cost = (double)((tiles + 255) / 256) * nj / eff;
    if (cost < best_cost - 1e-9) {
      best_cost = cost;
      best = nj;
    }
  }
  return best;
}

// Fused w1|w3 projection + SwiGLU (reference model.py:254 silu(w1 x) * w3 x): x [M, K],
// w13 = [w1; w3] [2F, K] -> (gu [M, 2F] = x w13^T for the backward, a = silu(g) u [M, F],
// a^T [F, M] for a weight gradient on transposed operands, empty when with_t is false).
// 32 NJ-column tiles: 16 NJ features of w1 and the same of w3 (nj = 0: pick_swiglu_nj);
// M % 256, F % (16 NJ), K % 128.
std::tuple<at::Tensor, at::Tensor, at::Tensor> gemm_swiglu_w4(const at::Tensor& x, const at::Tensor& w13,
                                                              bool with_t, int64_t nj) {
  FT_CHECK_CUDA(x);
  TORCH_CHECK(x.scalar_type() == at::kBFloat16 || x.scalar_type() == at::kHalf, "gemm_swiglu_w4: bf16 / fp16");
  TORCH_CHECK(w13.scalar_type() == x.scalar_type(), "gemm_swiglu_w4: x / w13 dtype mismatch");
  FT_CHECK_CONTIG(x);
  FT_CHECK_CONTIG(w13);
  const long M = x.size(0), K = x.size(1), F2 = w13.size(0), F = F2 / 2;
  const int NJ = nj > 0 ? (int)nj : pick_swiglu_nj(M, F), NWC = 16 * NJ;
  TORCH_CHECK(NJ == 8 || NJ == 7 || NJ == 6 || NJ == 4, "gemm_swiglu_w4: no tile width fits F = ", F);
  TORCH_CHECK(w13.size(1) == K && F2 % 2 == 0, "gemm_swiglu_w4: shape mismatch");
  TORCH_CHECK(M % BM == 0 && F % NWC == 0 && K % (2 * BK) == 0 && K > 0, "gemm_swiglu_w4: M % 256, F % ", NWC,
              ", K % 128 (got ", M, " ", F, " ", K, ")");
  TORCH_CHECK(M * K * 2 < (1L << 32) && F2 * K * 2 < (1L << 32), "gemm_swiglu_w4: operand over 4 GiB");
  const at::DeviceGuard guard(x.device());
  auto gu = at::empty({M, F2}, x.options());
  auto a = at::empty({M, F}, x.options());
  auto aT = with_t ? at::empty({F, M}, x.options()) : at::empty({0}, x.options());
  W4Args p{};
  p.prof = g_prof;
  p.group = raster_group(false);
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
  p.actT = with_t ? mptr<bf16_t>(aT) : nullptr;
  p.exact = (int)ft_exact_math();
  p.splits = 1;
  launch(x.scalar_type(), NJ, p, W4_SWIGLU, ft_stream());
  FT_LAUNCH_CHECK();
  return {gu, a, aT};
}

// FFN backward through w2 and the SwiGLU (reference model.py:254): da = dy [M, D] @ w2 [D, F]
// (w2 read as stored: k-major B), and in the epilogue dgu = [dg | du] from the saved gu [M, 2F]
// (swiglu_grad, as swiglu_bwd) — the separate SwiGLU-backward pass and da itself never exist.
at::Tensor gemm_swiglu_bwd_w4(const at::Tensor& dy, const at::Tensor& w2, const at::Tensor& gu, int64_t nj) {
  FT_CHECK_CUDA(dy);
  TORCH_CHECK(dy.scalar_type() == at::kBFloat16 || dy.scalar_type() == at::kHalf, "gemm_swiglu_bwd_w4: bf16 / fp16");
  TORCH_CHECK(w2.scalar_type() == dy.scalar_type() && gu.scalar_type() == dy.scalar_type(),
              "gemm_swiglu_bwd_w4: dtype mismatch");
  FT_CHECK_CONTIG(dy);
  FT_CHECK_CONTIG(w2);
  FT_CHECK_CONTIG(gu);
  const long D = w2.size(0), F = w2.size(1), M = dy.numel() / D;
  TORCH_CHECK(dy.numel() == M * D && gu.numel() == M * 2 * F, "gemm_swiglu_bwd_w4: shape mismatch");
  const int NJ = nj > 0 ? (int)nj : pick_nj(M, F);
  TORCH_CHECK(NJ == 8 || NJ == 7 || NJ == 6 || NJ == 4, "gemm_swiglu_bwd_w4: no tile width fits F = ", F);
  TORCH_CHECK(M % BM == 0 && F % (32 * NJ) == 0 && D % (2 * BK) == 0 && D > 0, "gemm_swiglu_bwd_w4: M % 256, F % ",
              32 * NJ, ", D % 128 (got ", M, " ", F, " ", D, ")");
  TORCH_CHECK(M * D * 2 < (1L << 32) && D * F * 2 < (1L << 32), "gemm_swiglu_bwd_w4: operand over 4 GiB");
  const at::DeviceGuard guard(dy.device());
  auto dgu = at::empty({M, 2 * F}, dy.options());
  W4Args p{};
  p.prof = g_prof;
  p.group = raster_group(false, 8);
  p.a = cptr<bf16_t>(dy);
  p.b = cptr<bf16_t>(w2);
  p.c = mptr<bf16_t>(dgu);
  p.r = cptr<bf16_t>(gu);
  p.lda = D;
  p.ldb = F;
  p.ldc = 2 * F;
  p.ldr = 2 * F;
  p.M = M;
  p.N = F;
  p.K = D;
  p.tiles_m = M / BM;
  p.tiles_n = F / (32 * NJ);
  p.nfast = 0;
  p.ffn = (int)F;
  p.exact = (int)ft_exact_math();
  p.splits = 1;
  launch(dy.scalar_type(), NJ, p, W4_SWIGLU_BWD, ft_stream(), false, true);
  FT_LAUNCH_CHECK();
  return dgu;
}

int64_t gemm_w4_pick(int64_t M, int64_t N) { return pick_nj(M, N); }
int64_t gemm_swiglu_pick(int64_t M, int64_t F) { return pick_swiglu_nj(M, F); }

// FT_W4_SPLITK at run time (A/B): 0 off, 1 automatic, 2 forced where it fits
void gemm_w4_set_splitk(int64_t mode) { g_splitk_mode = (int)mode; }

// Before a stream capture: the capture stream (current stream) gets its own split-K flag buffer,
// so the graph's split products keep their split (same summation order as the eager step) and
// never share flags with eager launches (graphs.GraphedStep.prime).
void gemm_w4_prepare_capture() {
  const auto cur = at::hip::getCurrentHIPStreamMasqueradingAsCUDA();
  std::lock_guard<std::mutex> lock(g_tick_mu);
  tick_buffer_locked(cur.device(), cur.stream());
}

// Split-K hand-offs that timed out since the last reset, summed over every flag buffer (a device
// sync per buffer: diagnostics / tests, not the step).
int64_t gemm_w4_splitk_errors(bool reset) {
  std::lock_guard<std::mutex> lock(g_tick_mu);
  int64_t n = 0;
  for (auto& kv : g_tick_bufs) {
    at::Tensor w = kv.second.narrow(0, TICKS - 1, 1);
    n += w.item<int>();
    if (reset) w.zero_();
  }
  return n;
}

// split-K consumer poll bound (tests of the timeout path; default 2^22)
void gemm_w4_set_spin(int64_t n) { g_spin = (int)std::max<int64_t>(1, n); }
void gemm_w4_set_deadzero(int64_t on) { g_deadzero = (int)on; }
void gemm_w4_set_remainder(int64_t on) { g_remainder = (int)on; }

// timing probes only (scripts/w4_overhead_probe.py): bit 0 skips the store / residual epilogues'
// global stores (the output is left unwritten)
void gemm_w4_set_dbg(int64_t v) { g_dbg = (int)v; }
void gemm_w4_set_group(int64_t v) { g_group = (int)v; }
void gemm_w4_set_prof(const std::optional<at::Tensor>& buf) {
  if (buf.has_value()) {
    TORCH_CHECK(buf->scalar_type() == at::kLong && buf->is_contiguous(), "gemm_w4_set_prof: int64 buffer");
    g_prof = reinterpret_cast<long long*>(buf->data_ptr<int64_t>());
    g_prof_rows = buf->numel() / 8;
  } else {
    g_prof = nullptr;
    g_prof_rows = 0;
  }
}

// (tile width / 32, splits) the automatic choice takes for C[M, N] over a K-deep sum
std::vector<int64_t> gemm_w4_plan(int64_t M, int64_t N, int64_t K, bool a_t, bool b_t) {
  const Plan pl = pick_plan(M, N, K, a_t, b_t);
  return {pl.nj, pl.splits};
}

TORCH_LIBRARY_FRAGMENT(ftamd, m) {
  m.def("gemm_nt_w4(Tensor a, Tensor b, Tensor(a!)? out=None, Tensor? residual=None, int nj=0, int splits=0) -> Tensor",
        &gemm_nt_w4);
  m.def(
      "gemm_w4_ex(Tensor a, bool a_t, Tensor b, bool b_t, int M, int N, int K, Tensor(a!)? out=None, "
      "bool accumulate=False, Tensor(b!)? part=None, int nj=0, int splits=0) -> Tensor",
      &gemm_w4_ex);
  m.def("gemm_w4_plan(int M, int N, int K, bool a_t=False, bool b_t=False) -> int[]", &gemm_w4_plan);
  m.def("gemm_w4_set_splitk(int mode) -> ()", &gemm_w4_set_splitk);
  m.def("gemm_w4_prepare_capture() -> ()", &gemm_w4_prepare_capture);
  m.def("gemm_w4_splitk_errors(bool reset=False) -> int", &gemm_w4_splitk_errors);
  m.def("gemm_w4_set_spin(int n) -> ()", &gemm_w4_set_spin);
  m.def("gemm_w4_set_deadzero(int on) -> ()", &gemm_w4_set_deadzero);
  m.def("gemm_w4_set_remainder(int on) -> ()", &gemm_w4_set_remainder);
  m.def("gemm_w4_set_dbg(int v) -> ()", &gemm_w4_set_dbg);
  m.def("gemm_w4_set_group(int v) -> ()", &gemm_w4_set_group);
  m.def("gemm_w4_set_prof(Tensor? buf) -> ()", &gemm_w4_set_prof);
  m.def("gemm_qkv_rope_w4(Tensor x, Tensor w, Tensor cos, Tensor sin, int seq, int hq, int hkv, int d) -> Tensor",
        &gemm_qkv_rope_w4);
  m.def("gemm_w4_pick(int M, int N) -> int", &gemm_w4_pick);
  m.def("gemm_swiglu_w4(Tensor x, Tensor w13, bool with_t=True, int nj=0) -> (Tensor, Tensor, Tensor)",
        &gemm_swiglu_w4);
  m.def("gemm_swiglu_pick(int M, int F) -> int", &gemm_swiglu_pick);
  m.def("gemm_swiglu_bwd_w4(Tensor dy, Tensor w2, Tensor gu, int nj=0) -> Tensor", &gemm_swiglu_bwd_w4);
}
