"""HIP flash attention (fwd + bwd) vs an fp32 PyTorch reference (repeat_kv + causal softmax)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def ref_attn(q, k, v):
    """q [B,S,Hq,D], k/v [B,S,Hkv,D] fp32 -> o [B,S,Hq,D]."""
    B, S, Hq, D = q.shape
    rep = Hq // k.shape[2]
    k = k.repeat_interleave(rep, 2)
    v = v.repeat_interleave(rep, 2)
    s = torch.einsum("bqhd,bkhd->bhqk", q, k) / D**0.5
    mask = torch.ones(S, S, dtype=torch.bool, device=q.device).triu(1)
    s = s.masked_fill(mask, float("-inf"))
    p = s.softmax(-1)
    return torch.einsum("bhqk,bkhd->bqhd", p, v)


def rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


@pytest.mark.parametrize(
    "B,S,Hq,Hkv,D",
    [(1, 128, 2, 1, 128), (1, 256, 4, 2, 128), (2, 192, 4, 4, 64), (1, 2048, 32, 8, 128), (1, 320, 8, 2, 64),
     (2, 512, 12, 12, 64),
     # long context (reduced heads) and sequence lengths that are not multiples of the 32/64/128 tiles
     (1, 8192, 4, 1, 128), (1, 1000, 4, 2, 128), (2, 2047, 2, 1, 64), (1, 33, 2, 2, 128), (3, 100, 4, 4, 64)],
)
@pytest.mark.parametrize("mode", [0, 1])
def test_flash_fwd_bwd(B, S, Hq, Hkv, D, mode):
    from fault_tolerant_llm_training_amd._native import kernels

    K = kernels()
    torch.manual_seed(0)
    T = B * S
    qkv = torch.randn(T, (Hq + 2 * Hkv) * D, device="cuda").bfloat16()
    qk = torch.randn(T, (Hq + Hkv) * D, device="cuda").bfloat16()
    o, lse = K.flash_fwd(qk, qkv, S, Hq, Hkv, D)
    q = qk[:, : Hq * D].float().view(B, S, Hq, D).requires_grad_(True)
    k = qk[:, Hq * D :].float().view(B, S, Hkv, D).requires_grad_(True)
    v = qkv[:, (Hq + Hkv) * D :].float().view(B, S, Hkv, D).requires_grad_(True)
    ref = ref_attn(q, k, v)
    assert rel(o.view(B, S, Hq, D), ref) < 1e-2
    do = torch.randn(T, Hq * D, device="cuda").bfloat16()
    dqkv = K.flash_bwd(do, qk, qkv, o, lse, S, Hq, Hkv, D, mode)
    gq, gk, gv = torch.autograd.grad(ref, (q, k, v), do.float().view(B, S, Hq, D))
    assert rel(dqkv[:, : Hq * D].view(B, S, Hq, D), gq) < 2e-2
    assert rel(dqkv[:, Hq * D : (Hq + Hkv) * D].view(B, S, Hkv, D), gk) < 2e-2
    assert rel(dqkv[:, (Hq + Hkv) * D :].view(B, S, Hkv, D), gv) < 2e-2


def test_flash_deterministic_fwd():
    from fault_tolerant_llm_training_amd._native import kernels

    K = kernels()
    qkv = torch.randn(1024, 48 * 128, device="cuda").bfloat16()
    qk = torch.randn(1024, 40 * 128, device="cuda").bfloat16()
    o1, _ = K.flash_fwd(qk, qkv, 1024, 32, 8, 128)
    o2, _ = K.flash_fwd(qk, qkv, 1024, 32, 8, 128)
    assert torch.equal(o1, o2)


def test_flash_bwd_deterministic_mode_is_bitwise_reproducible():
    from fault_tolerant_llm_training_amd._native import kernels

    K = kernels()
    torch.manual_seed(1)
    S, Hq, Hkv, D = 1024, 32, 8, 128
    qkv = torch.randn(S, (Hq + 2 * Hkv) * D, device="cuda").bfloat16()
    qk = torch.randn(S, (Hq + Hkv) * D, device="cuda").bfloat16()
    do = torch.randn(S, Hq * D, device="cuda").bfloat16()
    o, lse = K.flash_fwd(qk, qkv, S, Hq, Hkv, D)
    a = K.flash_bwd(do, qk, qkv, o, lse, S, Hq, Hkv, D, 1)
    b = K.flash_bwd(do, qk, qkv, o, lse, S, Hq, Hkv, D, 1)
    assert torch.equal(a, b)
    c = K.flash_bwd(do, qk, qkv, o, lse, S, Hq, Hkv, D, 0)
    assert ((a.float() - c.float()).norm() / c.float().norm()).item() < 1e-2


@pytest.mark.parametrize("slope", [0.02, 0.07, 0.3])
def test_flash_fwd_growing_scores(slope):
    """Scores that grow along the key axis at several rates, so the forward's running max moves
    by amounts around the deferred-rescale threshold on many tiles (rare on random data)."""
    from fault_tolerant_llm_training_amd._native import kernels

    K = kernels()
    torch.manual_seed(1)
    S, Hq, Hkv, D = 1024, 4, 2, 128
    q = torch.randn(S, Hq, D, device="cuda")
    u = torch.nn.functional.normalize(torch.randn(D, device="cuda"), dim=0)
    q = q + 4.0 * u  # every query has a component along u
    ramp = slope * torch.arange(S, device="cuda", dtype=torch.float32).view(S, 1, 1)
    k = 0.5 * torch.randn(S, Hkv, D, device="cuda") + ramp * u  # later keys score higher
    v = torch.randn(S, Hkv, D, device="cuda")
    qk = torch.cat([q.reshape(S, -1), k.reshape(S, -1)], 1).bfloat16()
    qkv = torch.cat([qk, v.reshape(S, -1).bfloat16()], 1)
    o, _ = K.flash_fwd(qk, qkv, S, Hq, Hkv, D)
    ref = ref_attn(qk[:, : Hq * D].float().view(1, S, Hq, D), qk[:, Hq * D :].float().view(1, S, Hkv, D),
                   v.bfloat16().float().view(1, S, Hkv, D))
    assert torch.isfinite(o).all()
    assert rel(o.view(1, S, Hq, D), ref) < 1e-2


@pytest.mark.parametrize("B,S,Hq,Hkv,D", [(1, 2048, 12, 12, 64), (2, 320, 8, 2, 128), (1, 100, 4, 4, 64),
                                         (1, 33, 2, 1, 128), (1, 4096, 4, 1, 128)])
def test_flash_fwd_key_split_matches(B, S, Hq, Hkv, D):
    """The key-split forward (two half-blocks over even / odd key tiles, merged in LDS) equals the
    one-pass forward up to summation order, incl. query tiles whose odd half sees no key, and its
    log-sum-exp drives the backward the same way."""
    from fault_tolerant_llm_training_amd._native import kernels

    K = kernels()
    torch.manual_seed(3)
    T = B * S
    qkv = torch.randn(T, (Hq + 2 * Hkv) * D, device="cuda").bfloat16()
    qk = torch.randn(T, (Hq + Hkv) * D, device="cuda").bfloat16()
    try:
        K.flash_set_fwd_split(0)
        o0, l0 = K.flash_fwd(qk, qkv, S, Hq, Hkv, D)
        K.flash_set_fwd_split(1)
        o1, l1 = K.flash_fwd(qk, qkv, S, Hq, Hkv, D)
    finally:
        K.flash_set_fwd_split(-1)
    assert torch.isfinite(o1).all()
    assert rel(o1, o0) < 4e-3
    Sp = l0.shape[-1]
    valid = torch.arange(Sp, device="cuda") < S
    assert (l1[..., valid] - l0[..., valid]).abs().max().item() < 1e-3
    do = torch.randn(T, Hq * D, device="cuda").bfloat16()
    g0 = K.flash_bwd(do, qk, qkv, o0, l0, S, Hq, Hkv, D, 1)
    g1 = K.flash_bwd(do, qk, qkv, o1, l1, S, Hq, Hkv, D, 1)
    assert rel(g1, g0) < 1e-2


@pytest.mark.parametrize("B,S,Hq,Hkv,D", [(1, 2048, 32, 8, 128), (2, 1000, 8, 2, 128), (3, 100, 4, 4, 64),
                                         (1, 33, 2, 1, 128), (1, 8192, 4, 1, 128), (2, 2047, 8, 8, 64),
                                         (1, 64, 2, 2, 64), (1, 65, 2, 1, 128)])
def test_flash_fwd_pipe_matches(B, S, Hq, Hkv, D):
    """The software-pipelined forward (next tile's scores issued with this tile's softmax) applies
    the same operations to O / l / m in the same order as the unpipelined kernel: bitwise equal."""
    from fault_tolerant_llm_training_amd._native import kernels

    K = kernels()
    torch.manual_seed(5)
    T = B * S
    qkv = torch.randn(T, (Hq + 2 * Hkv) * D, device="cuda").bfloat16()
    qk = torch.randn(T, (Hq + Hkv) * D, device="cuda").bfloat16()
    try:
        K.flash_set_fwd_split(0)
        K.flash_set_fwd_pipe(0)
        o0, l0 = K.flash_fwd(qk, qkv, S, Hq, Hkv, D)
        K.flash_set_fwd_pipe(2)
        o1, l1 = K.flash_fwd(qk, qkv, S, Hq, Hkv, D)
    finally:
        K.flash_set_fwd_split(-1)
        K.flash_set_fwd_pipe(1)
    valid = torch.arange(l0.shape[-1], device="cuda") < S
    assert torch.isfinite(o1).all()
    assert rel(o1, o0) < 1e-3
    assert (l1[..., valid] - l0[..., valid]).abs().max().item() < 1e-4
    q = qk[:, : Hq * D].float().view(B, S, Hq, D)
    k = qk[:, Hq * D :].float().view(B, S, Hkv, D)
    v = qkv[:, (Hq + Hkv) * D :].float().view(B, S, Hkv, D)
    if S <= 2048:
        assert rel(o1.view(B, S, Hq, D), ref_attn(q, k, v)) < 1e-2


@pytest.mark.parametrize("B,S,Hq,Hkv,D", [(1, 2048, 12, 12, 64), (2, 320, 8, 2, 128), (1, 100, 4, 4, 64),
                                         (1, 4096, 4, 1, 128)])
def test_flash_dq_key_split_matches(B, S, Hq, Hkv, D):
    """The key-split dQ kernel (two half-blocks, partials added in LDS in a fixed order) equals
    the one-pass dQ up to summation order and is bit-reproducible; dK / dV are untouched."""
    from fault_tolerant_llm_training_amd._native import kernels

    K = kernels()
    torch.manual_seed(4)
    T = B * S
    qkv = torch.randn(T, (Hq + 2 * Hkv) * D, device="cuda").bfloat16()
    qk = torch.randn(T, (Hq + Hkv) * D, device="cuda").bfloat16()
    do = torch.randn(T, Hq * D, device="cuda").bfloat16()
    o, lse = K.flash_fwd(qk, qkv, S, Hq, Hkv, D)
    try:
        K.flash_set_dq_split(0)
        g0 = K.flash_bwd(do, qk, qkv, o, lse, S, Hq, Hkv, D, 1)
        K.flash_set_dq_split(1)
        g1 = K.flash_bwd(do, qk, qkv, o, lse, S, Hq, Hkv, D, 1)
        g2 = K.flash_bwd(do, qk, qkv, o, lse, S, Hq, Hkv, D, 1)
    finally:
        K.flash_set_dq_split(-1)
    assert torch.equal(g1, g2)
    nq = Hq * D
    assert rel(g1[:, :nq], g0[:, :nq]) < 4e-3
    assert torch.equal(g1[:, nq:], g0[:, nq:])


@pytest.mark.parametrize("B,S,Hq,Hkv,D", [(1, 2048, 12, 12, 64), (1, 100, 4, 4, 64), (2, 320, 8, 2, 64)])
def test_flash_dkdv_split_matches(B, S, Hq, Hkv, D):
    """The split dK/dV kernel (two half-blocks over alternate query-slice pairs, partials added in
    LDS in a fixed order) equals the unsplit one up to summation order, bit-reproducibly."""
    from fault_tolerant_llm_training_amd._native import kernels

    K = kernels()
    torch.manual_seed(5)
    T = B * S
    qkv = torch.randn(T, (Hq + 2 * Hkv) * D, device="cuda").bfloat16()
    qk = torch.randn(T, (Hq + Hkv) * D, device="cuda").bfloat16()
    do = torch.randn(T, Hq * D, device="cuda").bfloat16()
    o, lse = K.flash_fwd(qk, qkv, S, Hq, Hkv, D)
    try:
        K.flash_set_kv_split(0)
        g0 = K.flash_bwd(do, qk, qkv, o, lse, S, Hq, Hkv, D, 1)
        K.flash_set_kv_split(1)
        g1 = K.flash_bwd(do, qk, qkv, o, lse, S, Hq, Hkv, D, 1)
        g2 = K.flash_bwd(do, qk, qkv, o, lse, S, Hq, Hkv, D, 1)
    finally:
        K.flash_set_kv_split(-1)
    assert torch.equal(g1, g2)
    nq = Hq * D
    assert torch.equal(g1[:, :nq], g0[:, :nq])  # dQ untouched
    assert rel(g1[:, nq:], g0[:, nq:]) < 4e-3


@pytest.mark.parametrize("B,S,Hq,Hkv,D,mode", [(1, 2048, 32, 8, 128, 1), (1, 512, 8, 2, 64, 1), (2, 256, 4, 4, 64, 1),
                                              (1, 1000, 4, 2, 128, 0), (2, 512, 12, 12, 64, 1),
                                              (1, 1024, 8, 8, 128, 1), (1, 300, 16, 16, 64, 1)])
def test_flash_bwd_with_rope_backward(B, S, Hq, Hkv, D, mode):
    """flash_bwd(..., cos, sin): the gradient of the UNROTATED projection, the RoPE backward done
    in the pass that folds the GQA partials, or -- no GQA -- in the dQ and dK/dV kernels' stores
    (round 6: no rope_bwd_ pass) == flash_bwd then rope_bwd_ (reference model.py:100-126) within one
    bf16 rounding; deterministic."""
    from fault_tolerant_llm_training_amd._native import kernels
    from fault_tolerant_llm_training_amd.models.llama import rope_tables

    K = kernels()
    torch.manual_seed(2)
    T = B * S
    qkv = torch.randn(T, (Hq + 2 * Hkv) * D, device="cuda").bfloat16()
    qk = torch.randn(T, (Hq + Hkv) * D, device="cuda").bfloat16()
    do = torch.randn(T, Hq * D, device="cuda").bfloat16()
    cos, sin = (t.cuda() for t in rope_tables(D, S, 500000.0))
    o, lse = K.flash_fwd(qk, qkv, S, Hq, Hkv, D)
    ref = K.flash_bwd(do, qk, qkv, o, lse, S, Hq, Hkv, D, mode)
    K.rope_bwd_(ref, cos, sin, S, Hq, Hkv, D)
    got = K.flash_bwd(do, qk, qkv, o, lse, S, Hq, Hkv, D, mode, cos, sin)
    for lo, hi in ((0, Hq * D), (Hq * D, (Hq + Hkv) * D), ((Hq + Hkv) * D, (Hq + 2 * Hkv) * D)):
        assert rel(got[:, lo:hi], ref[:, lo:hi]) < 4e-3, (lo, hi)
    if mode == 1:
        assert torch.equal(got, K.flash_bwd(do, qk, qkv, o, lse, S, Hq, Hkv, D, mode, cos, sin))


@pytest.mark.parametrize("B,S,Hq,Hkv,D,rope", [(1, 2048, 32, 8, 128, True), (2, 320, 8, 2, 128, False),
                                               (1, 1000, 4, 1, 128, True), (2, 512, 8, 2, 64, True),
                                               (1, 100, 6, 2, 64, False), (1, 512, 16, 1, 128, True)])
def test_flash_bwd_in_kernel_gqa_fold(B, S, Hq, Hkv, D, rope):
    """Deterministic backward, opt-in variant (flash_set_bwd_fold): the GQA fold (+ RoPE backward)
    done by the last q-head block of each key tile inside the dK/dV kernel == the finalize pass, bit
    for bit (same head order), and stays so over repeated launches (the counters re-arm)."""
    from fault_tolerant_llm_training_amd._native import kernels
    from fault_tolerant_llm_training_amd.models.llama import rope_tables

    K = kernels()
    torch.manual_seed(6)
    T = B * S
    qkv = torch.randn(T, (Hq + 2 * Hkv) * D, device="cuda").bfloat16()
    qk = torch.randn(T, (Hq + Hkv) * D, device="cuda").bfloat16()
    do = torch.randn(T, Hq * D, device="cuda").bfloat16()
    cs = tuple(t.cuda() for t in rope_tables(D, S, 500000.0)) if rope else (None, None)
    o, lse = K.flash_fwd(qk, qkv, S, Hq, Hkv, D)
    try:
        K.flash_set_bwd_fold(False)
        ref = K.flash_bwd(do, qk, qkv, o, lse, S, Hq, Hkv, D, 1, *cs)
        K.flash_set_bwd_fold(True)
        outs = [K.flash_bwd(do, qk, qkv, o, lse, S, Hq, Hkv, D, 1, *cs) for _ in range(3)]
    finally:
        K.flash_set_bwd_fold(False)
    for g in outs:
        assert torch.equal(g, ref)  # (G = 16 > 8: the fold is skipped, the finalize pass runs)


def test_flash_fwd_timing_probe():
    """flash_set_fwd_prof (scripts/flash_fwd_timeline.py): one row of ordered stamps per block, and
    the probed forward's output equals the unprobed one."""
    from fault_tolerant_llm_training_amd._native import kernels

    K = kernels()
    torch.manual_seed(9)
    S, Hq, Hkv, D = 1024, 8, 2, 128
    qkv = torch.randn(S, (Hq + 2 * Hkv) * D, device="cuda").bfloat16()
    qk = torch.randn(S, (Hq + Hkv) * D, device="cuda").bfloat16()
    buf = torch.zeros((S // 128) * Hq, 8, dtype=torch.int64, device="cuda")
    try:
        K.flash_set_fwd_split(0)  # the probe is in the pipelined (unsplit) kernel
        o0, _ = K.flash_fwd(qk, qkv, S, Hq, Hkv, D)
        K.flash_set_fwd_prof(buf)
        o1, _ = K.flash_fwd(qk, qkv, S, Hq, Hkv, D)
        torch.cuda.synchronize()
    finally:
        K.flash_set_fwd_prof(None)
        K.flash_set_fwd_split(-1)
    assert torch.equal(o0, o1)
    p = buf.cpu()
    assert (p[:, 0] > 0).all()
    assert (p[:, 1] >= p[:, 0]).all() and (p[:, 2] >= p[:, 1]).all() and (p[:, 3] >= p[:, 2]).all()
    assert sorted(set((p[:, 6] // 4).tolist())) == list(range(S // 128))
    small = torch.zeros(3, 8, dtype=torch.int64, device="cuda")  # fewer rows than blocks
    try:
        K.flash_set_fwd_split(0)
        K.flash_set_fwd_prof(small)
        with pytest.raises(RuntimeError, match="flash_set_fwd_prof"):
            K.flash_fwd(qk, qkv, S, Hq, Hkv, D)
    finally:
        K.flash_set_fwd_prof(None)
        K.flash_set_fwd_split(-1)


@pytest.mark.parametrize("S,H,D", [(512, 12, 64), (1024, 8, 128)])
def test_no_gqa_rope_in_kernel_matches_the_separate_pass(S, H, D):
    """No GQA: dQ / dK rotated back inside the two backward kernels (default) vs the separate
    rope_bwd_ pass after them (flash_set_direct_rope(False)): dQ rotated in fp32 before its one
    rounding (equal within bf16), dK rotated per 16-B chunk as rope_bwd_ does (bitwise), dV identical."""
    from fault_tolerant_llm_training_amd._native import kernels
    from fault_tolerant_llm_training_amd.models.llama import rope_tables

    K = kernels()
    torch.manual_seed(5)
    qkv = torch.randn(S, 3 * H * D, device="cuda").bfloat16()
    qk = torch.randn(S, 2 * H * D, device="cuda").bfloat16()
    do = torch.randn(S, H * D, device="cuda").bfloat16()
    cos, sin = (t.cuda() for t in rope_tables(D, S, 10000.0))
    o, lse = K.flash_fwd(qk, qkv, S, H, H, D)
    got = K.flash_bwd(do, qk, qkv, o, lse, S, H, H, D, 1, cos, sin)
    try:
        K.flash_set_direct_rope(False)
        sep = K.flash_bwd(do, qk, qkv, o, lse, S, H, H, D, 1, cos, sin)
    finally:
        K.flash_set_direct_rope(True)
    assert rel(got[:, : H * D], sep[:, : H * D]) < 4e-3
    assert torch.equal(got[:, H * D:], sep[:, H * D:])


@pytest.mark.parametrize("B,S,Hq,Hkv,D,rope", [(1, 2048, 32, 8, 128, True), (2, 320, 8, 2, 128, False),
                                               (1, 1000, 4, 1, 128, True), (2, 512, 8, 2, 64, True),
                                               (1, 100, 6, 2, 64, False), (1, 777, 16, 2, 128, True)])
def test_gqa_backward_in_three_kernels_equals_four(B, S, Hq, Hkv, D, rope):
    """GQA deterministic backward in 3 kernels (flash_set_fold3(True): dK/dV first forming delta from
    O, then dQ folding the per-q-head partials) == the default 4-kernel order (dQ, dK/dV, finalize),
    bit for bit: delta, the fold order and the RoPE arithmetic are term-for-term the same."""
    from fault_tolerant_llm_training_amd._native import kernels
    from fault_tolerant_llm_training_amd.models.llama import rope_tables

    K = kernels()
    torch.manual_seed(S + Hq)
    T = B * S
    qkv = torch.randn(T, (Hq + 2 * Hkv) * D, device="cuda").bfloat16()
    qk = torch.randn(T, (Hq + Hkv) * D, device="cuda").bfloat16()
    do = torch.randn(T, Hq * D, device="cuda").bfloat16()
    cs = tuple(t.cuda() for t in rope_tables(D, S, 500000.0)) if rope else (None, None)
    o, lse = K.flash_fwd(qk, qkv, S, Hq, Hkv, D)
    four = K.flash_bwd(do, qk, qkv, o, lse, S, Hq, Hkv, D, 1, *cs)
    try:
        K.flash_set_fold3(True)
        three = K.flash_bwd(do, qk, qkv, o, lse, S, Hq, Hkv, D, 1, *cs)
    finally:
        K.flash_set_fold3(False)
    assert torch.equal(three, four), (three.float() - four.float()).abs().max().item()
