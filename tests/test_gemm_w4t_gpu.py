"""The w4 GEMM on k-major operands (csrc/kernels/gemm_w4.hip: ds_read_b64_tr_b16 images) vs fp32.

dX layout  C = A B        A [M, K] as stored, B stored [K, N]          (dY [T, N] @ W [N, K])
dW layout  C = A^T B      A stored [K, M], B stored [K, N]            (dY^T [N, T] @ X [T, K])
Every tile width (NJ 4 / 6 / 7 / 8: the four k-major row lengths and their swizzles), both
rasters, the accumulate and sum-of-squares epilogues, the fused SwiGLU backward, fp16, and the
Llama-3-8B product shapes. Integer-valued operands make the fp32 reference exact, so those
checks are bitwise (any swizzle / lane-map error moves whole values); random operands check the
relative error. Reference math: model.py:195,215,254,379 and their gradients.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu


def K():
    from fault_tolerant_llm_training_amd._native import kernels

    return kernels()


def ints(*s, lo=-3, hi=4, dtype=torch.bfloat16):
    return torch.randint(lo, hi, s, device="cuda").to(dtype)


def rnd(*s, dtype=torch.bfloat16):
    return (torch.rand(*s, device="cuda") * 2 - 1).to(dtype)


def rel(out, ref):
    return ((out.float() - ref).norm() / ref.norm()).item()


@pytest.mark.parametrize("nj", [4, 6, 7, 8])
@pytest.mark.parametrize("M,Kd", [(256, 128), (512, 384), (768, 1024)])
def test_dx_layout_exact(nj, M, Kd):
    torch.manual_seed(nj * 7 + M + Kd)
    N = 32 * nj * 3
    a = ints(M, Kd)
    b = ints(Kd, N) + (torch.arange(N, device="cuda") % 5).bfloat16()  # asymmetric columns
    out = K().gemm_w4_ex(a, False, b, True, M, N, Kd, None, False, None, nj)
    ref = (a.float() @ b.float()).bfloat16()
    assert torch.equal(out, ref), (out.float() - ref.float()).abs().max().item()


@pytest.mark.parametrize("nj", [4, 6, 7, 8])
@pytest.mark.parametrize("M,Kd", [(256, 128), (512, 256), (768, 2048)])
def test_dw_layout_exact(nj, M, Kd):
    torch.manual_seed(nj * 11 + M + Kd)
    N = 32 * nj * 2
    at = ints(Kd, M) + (torch.arange(M, device="cuda") % 3).bfloat16()  # A stored transposed
    b = ints(Kd, N)
    out = K().gemm_w4_ex(at, True, b, True, M, N, Kd, None, False, None, nj)
    ref = (at.float().t() @ b.float()).bfloat16()
    assert torch.equal(out, ref), (out.float() - ref.float()).abs().max().item()


@pytest.mark.parametrize("a_t", [False, True])
@pytest.mark.parametrize("M,N,Kd", [(1024, 256, 512), (256, 1792, 384)])
def test_both_rasters(a_t, M, N, Kd):
    """M > N rasters N-fastest inside an XCD's range, M < N M-fastest: same result either way."""
    torch.manual_seed(M + N)
    a = rnd(Kd, M) if a_t else rnd(M, Kd)
    b = rnd(Kd, N)
    out = K().gemm_w4_ex(a, a_t, b, True, M, N, Kd, None, False, None, 0)
    ref = (a.float().t() if a_t else a.float()) @ b.float()
    assert rel(out, ref) < 4e-3


@pytest.mark.parametrize("a_t", [False, True])
def test_accumulate_and_sumsq(a_t):
    torch.manual_seed(3)
    M, N, Kd = 512, 896, 256
    a = rnd(Kd, M) if a_t else rnd(M, Kd)
    b = rnd(Kd, N)
    ref = (a.float().t() if a_t else a.float()) @ b.float()
    nj = K().gemm_w4_pick(M, N)
    tiles = (M // 256) * (N // (32 * nj))
    part = torch.full((tiles + 5,), -1.0, device="cuda")
    c = rnd(M, N)
    c0 = c.float().clone()
    K().gemm_w4_ex(a, a_t, b, True, M, N, Kd, c, True, part, 0)
    assert rel(c, ref + c0) < 4e-3
    # one partial per tile, the sum of squares of exactly the stored (rounded) values
    assert torch.all(part[tiles:] == 0.0)  # slots past the tile grid are zeroed (no stale partials)
    want = c.float().pow(2).sum().item()
    got = part[:tiles].double().sum().item()
    assert abs(got - want) <= 1e-5 * want, (got, want)
    # deterministic: same partials bit for bit
    part2 = torch.zeros(tiles, device="cuda")
    c2 = c0.bfloat16()
    K().gemm_w4_ex(a, a_t, b, True, M, N, Kd, c2, True, part2, 0)
    assert torch.equal(c2, c) and torch.equal(part2, part[:tiles])


@pytest.mark.parametrize("T,D,F", [(256, 256, 224), (512, 768, 1792), (2048, 4096, 14336)])
def test_swiglu_bwd_epilogue(T, D, F):
    """dgu from the fused kernel == swiglu_bwd(da) with da from the same GEMM (bitwise), and the
    fp32 SwiGLU derivative (reference model.py:254) within bf16 error."""
    torch.manual_seed(T + F)
    dy = rnd(T, D)
    w2 = (rnd(D, F) / D ** 0.5).bfloat16()
    gu = rnd(T, 2 * F) * 2
    nj = K().gemm_w4_pick(T, F)
    dgu = K().gemm_swiglu_bwd_w4(dy, w2, gu, 0)
    da = K().gemm_w4_ex(dy, False, w2, True, T, F, D, None, False, None, nj)
    assert torch.equal(dgu, K().swiglu_bwd(da, gu))
    g, u = gu.float()[:, :F], gu.float()[:, F:]
    daf = (dy.float() @ w2.float()).bfloat16().float()
    s = torch.sigmoid(g)
    ref = torch.cat([daf * u * (s + g * s * (1 - s)), daf * g * s], 1)
    assert rel(dgu, ref) < 1e-2


def test_k_must_pair():
    """K-tiles run in pairs (static LDS stage offsets): K % 128 is checked, not silently wrong."""
    a, b = rnd(256, 192), rnd(192, 256)
    with pytest.raises(RuntimeError, match="K % 128"):
        K().gemm_w4_ex(a, False, b, True, 256, 256, 192, None, False, None, 0)


def test_fp16_layouts():
    torch.manual_seed(5)
    M, N, Kd = 512, 512, 384
    a, b = rnd(M, Kd, dtype=torch.float16), rnd(Kd, N, dtype=torch.float16)
    out = K().gemm_w4_ex(a, False, b, True, M, N, Kd, None, False, None, 0)
    assert out.dtype == torch.float16 and rel(out, a.float() @ b.float()) < 2e-3
    at = rnd(Kd, M, dtype=torch.float16)
    out = K().gemm_w4_ex(at, True, b, True, M, N, Kd, None, False, None, 0)
    assert rel(out, at.float().t() @ b.float()) < 2e-3


# the Llama-3-8B backward products (T = 2048): dX of qkv / wo / w13, dW of qkv / wo / w13 / w2
@pytest.mark.parametrize("a_t,M,N,Kd", [(False, 2048, 4096, 6144), (False, 2048, 4096, 4096),
                                        (False, 2048, 4096, 28672), (True, 6144, 4096, 2048),
                                        (True, 4096, 4096, 2048), (True, 28672, 4096, 2048),
                                        (True, 4096, 14336, 2048)])
def test_llama8b_products(a_t, M, N, Kd):
    torch.manual_seed(M + N + Kd)
    a = rnd(Kd, M) if a_t else rnd(M, Kd)
    b = rnd(Kd, N)
    out = K().gemm_w4_ex(a, a_t, b, True, M, N, Kd, None, False, None, 0)
    ref = (a.float().t() if a_t else a.float()) @ b.float()
    assert rel(out, ref) < 4e-3


# ---- split-K (gemm_w4.h W4Args::splits): the two halves of K of a tile on two workgroups, the
# first half's fp32 partial added by the second in its epilogue (fixed order: deterministic)
@pytest.mark.parametrize("layout", ["fwd", "dx"])
@pytest.mark.parametrize("nj,M,N,Kd", [(8, 512, 512, 512), (8, 256, 768, 2048), (4, 512, 384, 1024),
                                       (7, 256, 448, 768)])
def test_split_k_exact_and_deterministic(layout, nj, M, N, Kd):
    torch.manual_seed(M + N + Kd + nj)
    a = ints(M, Kd)
    if layout == "fwd":
        b = ints(N, Kd)  # [N, K]: C = A B^T
        ref = a.float() @ b.float().t()
        run = lambda sp, out=None, acc=False: K().gemm_nt_w4(a, b, out, out if acc else None, nj, sp)  # noqa: E731
    else:
        b = ints(Kd, N)  # stored [K, N]: C = A B
        ref = a.float() @ b.float()
        run = lambda sp, out=None, acc=False: K().gemm_w4_ex(a, False, b, True, M, N, Kd, out, acc, None, nj, sp)  # noqa: E731
    c1, c2 = run(1), run(2)
    assert torch.equal(c2.float(), ref.bfloat16().float())  # integer sums: exact whatever the split
    assert torch.equal(c1, c2)
    # random operands: within bf16 rounding of fp32, and bitwise the same on every launch
    a.copy_(rnd(M, Kd))
    b.copy_(rnd(*b.shape))
    ref = a.float() @ (b.float().t() if layout == "fwd" else b.float())
    outs = [run(2) for _ in range(3)]
    assert rel(outs[0], ref) < 4e-3
    for o in outs[1:]:
        assert torch.equal(o, outs[0])
    # residual / accumulate epilogue on the split path
    c = rnd(M, N)
    c0 = c.float().clone()
    run(2, c, True)
    assert rel(c, ref + c0) < 4e-3


def test_split_k_plan_for_the_8b_dx_products():
    """The automatic plan splits the 8B dX products whose 256-wide tiles fill half the chip (N_out =
    4096 at M = 2048) and leaves the others alone."""
    T, D, F, V = 2048, 4096, 14336, 131072
    plan = lambda M, N, Kd, at=False, bt=True: list(K().gemm_w4_plan(M, N, Kd, at, bt))  # noqa: E731
    assert plan(T, D, 2 * F) == [8, 2]      # w13 dX
    assert plan(T, D, V) == [8, 2]          # LM-head dX
    assert plan(V, D, T, True, True)[1] == 1   # dW: never split
    assert plan(T, F, D)[1] == 1            # w2 dX: 512 tiles already


def test_split_k_8b_head_dx_vs_fp32():
    """The LM-head dX at the 8B shape (K = 131072 split in two halves of 65536) vs fp32."""
    torch.manual_seed(9)
    M, N, Kd = 2048, 4096, 131072
    a = rnd(M, Kd)
    b = rnd(Kd, N)
    c = K().gemm_w4_ex(a, False, b, True, M, N, Kd, None, False, None, 8, 2)
    rows = torch.arange(0, M, 97, device="cuda")
    ref = a[rows].float() @ b.float()
    assert rel(c[rows], ref) < 4e-3
    assert torch.equal(c, K().gemm_w4_ex(a, False, b, True, M, N, Kd, None, False, None, 8, 2))


@pytest.mark.parametrize("M", [768, 1160, 50304])
@pytest.mark.parametrize("nj,splits", [(4, 1), (4, 2), (4, 3), (4, 4), (8, 1), (6, 1)])
def test_dw_split_k_and_tail_tile(M, nj, splits):
    """The dW layout (k-major A and B) split over K (the GPT-2-sized weight gradients: 18-96 tiles of
    256 x 128 at 2048 tokens) and with a tail tile (M % 256 != 0: the GPT-2 LM-head dW at V = 50304):
    exact on integer operands for every split, the rows past M untouched, the sum-of-squares partials
    of the stored values only, the accumulate epilogue, and fp32-close on random operands."""
    k = K()
    torch.manual_seed(M + splits + nj)
    N, T = 768, 2048
    if M == 50304 and splits not in (1, 3):
        pytest.skip("the 50304 tail at two splits is enough")
    at = ints(T, M) + (torch.arange(M, device="cuda") % 3).bfloat16()  # dY [T, M] read k-major
    b = ints(T, N)
    ref = at.float().t() @ b.float()
    tiles = ((M + 255) // 256) * (N // (32 * nj))
    part = torch.full((tiles + 5,), 7.0, device="cuda")  # slots past the grid are zeroed
    big = torch.full((M + 64, N), 3.0, dtype=torch.bfloat16, device="cuda")  # rows past M: canary
    out = big[:M]
    k.gemm_w4_ex(at, True, b, True, M, N, T, out, False, part, nj, splits)
    assert torch.equal(out.float(), ref.bfloat16().float())
    assert (big[M:] == 3.0).all()
    assert part[tiles:].abs().sum().item() == 0
    sq = (out.float() ** 2).sum().item()
    assert abs(part.sum().item() - sq) <= 1e-5 * sq
    k.gemm_w4_ex(at, True, b, True, M, N, T, out, True, None, nj, splits)  # accumulate
    assert torch.equal(out.float(), (2 * ref).bfloat16().float())
    # random operands: fp32-close, bitwise reproducible, and split == unsplit within rounding
    at.copy_(rnd(T, M))
    b.copy_(rnd(T, N))
    ref = at.float().t() @ b.float()
    o1 = k.gemm_w4_ex(at, True, b, True, M, N, T, None, False, None, nj, splits)
    o2 = k.gemm_w4_ex(at, True, b, True, M, N, T, None, False, None, nj, splits)
    assert rel(o1, ref) < 4e-3 and torch.equal(o1, o2)


def test_gpt2_plans_split_the_small_dw_grids():
    """The automatic plan splits the GPT-2-sized weight gradients (128-wide tiles, K = 2048 tokens)
    and the tail-tile head dW at V = 50304 gets a plan at all."""
    plan = lambda M, N, Kd, at=True, bt=True: list(K().gemm_w4_plan(M, N, Kd, at, bt))  # noqa: E731
    for M, N in [(2304, 768), (768, 768), (4096, 768), (768, 2048), (3072, 1024), (1024, 1024)]:
        nj, sp = plan(M, N, 2048)
        assert nj == 4 and sp > 1, (M, N, nj, sp)
    assert plan(50304, 768, 2048)[0] > 0
    assert plan(131072, 4096, 2048) == [8, 1]  # the 8B head dW: a full grid, unsplit


@pytest.mark.parametrize("layout", ["fwd", "dx"])
def test_split_k_lost_handoff_is_loud(layout):
    """A split-K hand-off that never completes (test mode: the producers never raise their flags,
    the consumer's poll bound lowered) is counted in the error word and writes NaN for the whole
    tile -- the step's non-finite guard then skips the update -- instead of a silently wrong sum;
    the flags it never saw raised are not re-armed, and the next normal launch is exact again."""
    k = K()
    torch.manual_seed(5)
    M, N, Kd = 512, 512, 1024
    a = ints(M, Kd)
    if layout == "fwd":
        b = ints(N, Kd)
        ref = (a.float() @ b.float().t()).bfloat16()
        run = lambda: k.gemm_nt_w4(a, b, None, None, 8, 2)  # noqa: E731
    else:
        b = ints(Kd, N)
        ref = (a.float() @ b.float()).bfloat16()
        run = lambda: k.gemm_w4_ex(a, False, b, True, M, N, Kd, None, False, None, 8, 2)  # noqa: E731
    k.gemm_w4_splitk_errors(True)
    try:
        k.gemm_w4_set_spin(64)
        k.gemm_w4_set_dbg(2)
        bad = run()
        torch.cuda.synchronize()
    finally:
        k.gemm_w4_set_dbg(0)
        k.gemm_w4_set_spin(1 << 22)
    assert torch.isnan(bad.float()).all()
    assert k.gemm_w4_splitk_errors(True) == (M // 256) * (N // 256)
    assert torch.equal(run(), ref)
    assert k.gemm_w4_splitk_errors(False) == 0


def test_w4_timing_probe():
    """gemm_w4_set_prof (scripts/w4_timeline.py): one exit stamp per workgroup, output unchanged."""
    k = K()
    torch.manual_seed(11)
    M, N, Kd = 1024, 1024, 512
    a = torch.randint(-2, 3, (Kd, M), device="cuda").bfloat16()
    b = torch.randint(-2, 3, (Kd, N), device="cuda").bfloat16()
    c0 = k.gemm_w4_ex(a, True, b, True, M, N, Kd, None, False, None, 8, 1)
    buf = torch.zeros((M // 256) * (N // 256), 8, dtype=torch.int64, device="cuda")
    try:
        k.gemm_w4_set_prof(buf)
        c1 = k.gemm_w4_ex(a, True, b, True, M, N, Kd, None, False, None, 8, 1)
        torch.cuda.synchronize()
    finally:
        k.gemm_w4_set_prof(None)
    assert torch.equal(c0, c1)
    p = buf.cpu()
    assert (p[:, 3] > 0).all()
    assert sorted(p[:, 6].tolist()) == list(range(buf.shape[0]))
    small = torch.zeros(3, 8, dtype=torch.int64, device="cuda")  # fewer rows than workgroups
    try:
        k.gemm_w4_set_prof(small)
        with pytest.raises(RuntimeError, match="gemm_w4_set_prof"):
            k.gemm_w4_ex(a, True, b, True, M, N, Kd, None, False, None, 8, 1)
    finally:
        k.gemm_w4_set_prof(None)


@pytest.mark.parametrize("group", [2, 3, 4, 8])
def test_w4_grouped_raster_bitwise(group):
    """gemm_w4_set_group: a different tile -> workgroup order only; every layout, split-K and the
    sum-of-squares partials are bitwise the default raster's (incl. a last band shorter than G)."""
    k = K()
    torch.manual_seed(13)
    cases = []
    a, b = rnd(2048, 1024), rnd(1792, 1024)  # fwd: 8 x 14 tiles at NJ 4
    cases.append(lambda: (k.gemm_nt_w4(a, b, None, None),))
    a2, b2 = rnd(1280, 4096), rnd(4096, 1024)  # dX, split-K picked by the plan
    cases.append(lambda: (k.gemm_w4_ex(a2, False, b2, True, 1280, 1024, 4096, None, False, None, 0),))
    a3, b3 = rnd(512, 2816), rnd(512, 768)  # dW with partials: 11 x 3 tiles (M > N: n fastest)
    part = torch.zeros(11 * 6, device="cuda")

    def dw():
        part.zero_()
        c = k.gemm_w4_ex(a3, True, b3, True, 2816, 768, 512, None, False, part, 0)
        return c, part.clone()

    cases.append(dw)
    x, w13 = rnd(1024, 512), rnd(2 * 896, 512)
    cases.append(lambda: k.gemm_swiglu_w4(x, w13, True))
    ref = [f() for f in cases]
    try:
        k.gemm_w4_set_group(group)
        got = [f() for f in cases]
    finally:
        k.gemm_w4_set_group(-1)
    for r_, g_ in zip(ref, got):
        for u, v in zip(r_, g_):
            assert torch.equal(u, v)


def test_dead_tail_dmas_change_nothing():
    """gemm_w4_set_deadzero (FT_W4_DEADZERO): the last two K-tiles' LDS-DMAs (no tile t + 2 to fetch)
    through null descriptors (zeros into the dead stage, no memory traffic) or re-staging the last
    K-tile: bitwise the same products in every layout, split-K and epilogue."""
    k = K()
    torch.manual_seed(21)
    a, b = rnd(1024, 1024), rnd(768, 1024)
    a2, b2 = rnd(512, 4096), rnd(4096, 1024)
    at, x = rnd(2048, 2304), rnd(2048, 768)
    part = torch.zeros(64, device="cuda")
    cases = [lambda: k.gemm_nt_w4(a, b, None, None, 0, 0),
             lambda: k.gemm_w4_ex(a2, False, b2, True, 512, 1024, 4096, None, False, None, 8, 2),
             lambda: (k.gemm_w4_ex(at, True, x, True, 2304, 768, 2048, None, False, part, 4, 3), part.clone()),
             lambda: k.gemm_swiglu_w4(a, rnd(2 * 448, 1024), False)[:2]]
    torch.manual_seed(22)
    ref = [f() for f in cases]
    try:
        k.gemm_w4_set_deadzero(0)
        torch.manual_seed(22)
        got = [f() for f in cases]
    finally:
        k.gemm_w4_set_deadzero(1)
    for r_, g_ in zip(ref, got):
        for u, v in zip(r_ if isinstance(r_, tuple) else (r_,), g_ if isinstance(g_, tuple) else (g_,)):
            assert torch.equal(u, v)


def test_round_remainder_split_bitwise():
    """gemm_w4_set_remainder (FT_W4_REMAINDER): a dW grid of one full round plus half a round (the 8B
    qkv dW, 24 x 16 tiles of 256^2) runs as two launches over disjoint rows, the remainder at the
    128-wide tile. Same summation order per element: bitwise the single launch; the partial sums of
    squares cover the same values; accumulate too."""
    k = K()
    torch.manual_seed(31)
    M, N, T = 6144, 4096, 2048
    at, x = rnd(T, M), rnd(T, N)
    part = torch.zeros(768, device="cuda")

    def go():
        part.fill_(5.0)
        c = k.gemm_w4_ex(at, True, x, True, M, N, T, None, False, part, 0, 0)
        c2 = c.clone()
        k.gemm_w4_ex(at, True, x, True, M, N, T, c2, True, None, 0, 0)
        return c, c2, part.double().sum().item(), part[512:].abs().sum().item()

    c_on, acc_on, sq_on, rest_on = go()
    try:
        k.gemm_w4_set_remainder(0)
        c_off, acc_off, sq_off, rest_off = go()
    finally:
        k.gemm_w4_set_remainder(1)
    assert torch.equal(c_on, c_off) and torch.equal(acc_on, acc_off)
    assert rest_on == 0 and abs(sq_on - sq_off) <= 1e-5 * sq_off
    want = c_on.float().pow(2).sum().item()
    assert abs(sq_on - want) <= 1e-5 * want
