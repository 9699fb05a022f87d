"""The fp32 MFMA GEMM (csrc/kernels/gemm_f32.hip, v_mfma_f32_16x16x4_f32) vs a float64 reference.

C[M, N] (+)= A B^T over K with A, B in the three layouts of a linear layer's products (forward
x W^T, dX = dY W, dW = dY^T X) plus the fourth combination; M / N tails (partial 128 x 128 tiles);
the accumulate, residual and sum-of-squares epilogues; and an fp32 model's training step through
ops/functional.py against the hipBLASLt routing (set_f32_mfma(False)). Integer-valued operands make
the reference exact (bitwise checks: a lane-map or image-layout error moves whole values); random
operands check the relative error. Reference math: model.py:195,215,254,379, utils.py:14-19.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu


def K():
    from fault_tolerant_llm_training_amd._native import kernels

    return kernels()


def operands(M, N, Kd, a_t, b_t, ints):
    g = torch.Generator(device="cuda").manual_seed(M * 31 + N * 7 + Kd + 2 * a_t + b_t)
    if ints:
        mk = lambda *s: torch.randint(-4, 5, s, device="cuda", generator=g).float()  # noqa: E731
    else:
        mk = lambda *s: torch.rand(*s, device="cuda", generator=g) * 2 - 1  # noqa: E731
    a = mk(Kd, M) if a_t else mk(M, Kd)
    b = mk(Kd, N) if b_t else mk(N, Kd)
    A = a.t() if a_t else a
    B = b if b_t else b.t()  # [K, N]
    return a, b, A.double() @ B.double()


LAYOUTS = [(False, False), (False, True), (True, True), (True, False)]


@pytest.mark.parametrize("a_t,b_t", LAYOUTS)
@pytest.mark.parametrize("M,N,Kd", [(128, 128, 32), (256, 384, 160), (200, 72, 64), (516, 260, 96)])
def test_exact_integer_operands(a_t, b_t, M, N, Kd):
    a, b, ref = operands(M, N, Kd, a_t, b_t, True)
    out = K().gemm_f32(a, a_t, b, b_t, M, N, Kd)
    assert out.shape == (M, N)
    assert torch.equal(out.double(), ref), (out.double() - ref).abs().max().item()


@pytest.mark.parametrize("a_t,b_t", LAYOUTS)
@pytest.mark.parametrize("M,N,Kd", [(2048, 768, 768), (768, 2304, 2048), (1000, 1028, 4096)])
def test_random_operands_relative_error(a_t, b_t, M, N, Kd):
    a, b, ref = operands(M, N, Kd, a_t, b_t, False)
    out = K().gemm_f32(a, a_t, b, b_t, M, N, Kd)
    err = ((out.double() - ref).norm() / ref.norm()).item()
    assert err < 2e-6, err


def test_accumulate_residual_and_partials():
    M, N, Kd = 384, 640, 256
    a, b, ref = operands(M, N, Kd, True, True, True)
    c0 = torch.randint(-9, 10, (M, N), device="cuda").float()
    out = c0.clone()
    tiles = 3 * 5
    part = torch.full((tiles + 7,), 123.0, device="cuda")
    r = K().gemm_f32(a, True, b, True, M, N, Kd, out, True, part)
    assert r.data_ptr() == out.data_ptr()
    want = c0.double() + ref
    assert torch.equal(out.double(), want)
    # one partial per 128 x 128 tile at part[tn * tiles_m + tm], the slots past the grid zeroed
    sq = want.pow(2).reshape(3, 128, 5, 128).sum(dim=(1, 3))  # [tm, tn]
    assert torch.allclose(part[:tiles].double(), sq.t().reshape(-1), rtol=1e-6)
    assert torch.equal(part[tiles:], torch.zeros(7, device="cuda"))
    # residual (the forward layout's fused residual add)
    x, w, ref2 = operands(M, N, Kd, False, False, True)
    res = torch.randint(-9, 10, (M, N), device="cuda").float()
    y = K().gemm_f32(x, False, w, False, M, N, Kd, None, False, None, res)
    assert torch.equal(y.double(), ref2 + res.double())


def test_bad_shapes_are_refused():
    a = torch.zeros(128, 48, device="cuda")
    with pytest.raises(RuntimeError, match="multiple of 32"):
        K().gemm_f32(a, False, torch.zeros(128, 48, device="cuda"), False, 128, 128, 48)
    with pytest.raises(RuntimeError, match="M % 4"):
        K().gemm_f32(torch.zeros(64, 130, device="cuda"), True, torch.zeros(64, 128, device="cuda"), True,
                     130, 128, 64)


def test_fp32_model_step_matches_the_hipblaslt_routing():
    """A tiny fp32 model's loss and every gradient with the GEMMs on gemm_f32 vs on hipBLASLt."""
    from fault_tolerant_llm_training_amd.models.llama import build_model, model_args_for
    from fault_tolerant_llm_training_amd.ops import functional as Fx

    a = model_args_for("tiny", vocab_size=512, seq_len=128)
    tok = torch.randint(0, 512, (2, 128), device="cuda")
    lab = torch.randint(0, 512, (2, 128), device="cuda")
    out = {}
    for on in (True, False):
        Fx.set_f32_mfma(on)
        try:
            m = build_model(a, "cuda:0", torch.float32, seed=0)
            loss = m(tok, lab)
            loss.backward()
            torch.cuda.synchronize()
            out[on] = (loss.item(), m.flat.grads.clone())
        finally:
            Fx.set_f32_mfma(True)
    assert abs(out[True][0] - out[False][0]) < 1e-5 * abs(out[False][0])
    g1, g0 = out[True][1], out[False][1]
    assert ((g1 - g0).norm() / g0.norm()).item() < 1e-5


@pytest.mark.parametrize("a_t,b_t", LAYOUTS)
def test_split_k_exact_and_epilogues(a_t, b_t):
    """Forced K slices (gemm_f32_set_splitk): integer operands stay exact; accumulate, residual and
    the per-tile partials come from the reduction pass."""
    M, N, Kd = 260, 384, 512
    a, b, ref = operands(M, N, Kd, a_t, b_t, True)
    k = K()
    try:
        for s in (2, 3, 8):
            k.gemm_f32_set_splitk(s)
            out = k.gemm_f32(a, a_t, b, b_t, M, N, Kd)
            assert torch.equal(out.double(), ref), (s, (out.double() - ref).abs().max().item())
        k.gemm_f32_set_splitk(4)
        c0 = torch.randint(-9, 10, (M, N), device="cuda").float()
        out = c0.clone()
        part = torch.full((3 * 3 + 5,), 7.0, device="cuda")
        k.gemm_f32(a, a_t, b, b_t, M, N, Kd, out, True, part)
        want = c0.double() + ref
        assert torch.equal(out.double(), want)
        sq = torch.zeros(3, 3, dtype=torch.float64, device="cuda")
        for tm in range(3):
            for tn in range(3):
                sq[tm, tn] = want[tm * 128:(tm + 1) * 128, tn * 128:(tn + 1) * 128].pow(2).sum()
        assert torch.allclose(part[:9].double(), sq.t().reshape(-1), rtol=1e-6)
        assert torch.equal(part[9:], torch.zeros(5, device="cuda"))
        res = torch.randint(-9, 10, (M, N), device="cuda").float()
        y = k.gemm_f32(a, a_t, b, b_t, M, N, Kd, None, False, None, res)
        assert torch.equal(y.double(), ref + res.double())
    finally:
        k.gemm_f32_set_splitk(-1)


def test_split_plan_fills_the_chip():
    """Automatic slices: none from 256 tiles; the GPT-2-sized 96-tile products split (>= 256 deep)."""
    k = K()
    assert k.gemm_f32_slices(2048, 28672, 4096) == 1
    assert k.gemm_f32_slices(2048, 768, 3072) > 1
    assert k.gemm_f32_slices(2048, 768, 4096) * 96 <= 512
    assert k.gemm_f32_slices(2048, 768, 128) == 1  # too shallow to split


@pytest.mark.parametrize("a_t,b_t", LAYOUTS)
def test_register_form_matches_the_dma_form(a_t, b_t):
    """The register round-trip form (gemm_f32_set_dma(0): operands larger than 32-bit buffer offsets)
    and the LDS-DMA form give the same exact products, tails included."""
    M, N, Kd = 516, 260, 192
    a, b, ref = operands(M, N, Kd, a_t, b_t, True)
    k = K()
    try:
        outs = []
        for dma in (1, 0):
            k.gemm_f32_set_dma(dma)
            outs.append(k.gemm_f32(a, a_t, b, b_t, M, N, Kd))
    finally:
        k.gemm_f32_set_dma(1)
    assert torch.equal(outs[0].double(), ref) and torch.equal(outs[1].double(), ref)
