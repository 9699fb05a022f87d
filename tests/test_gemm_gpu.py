"""Hand-written gfx950 GEMM (csrc/kernels/gemm.hip) vs an fp32 PyTorch reference.

Every operand layout the step uses (forward A_K/B_K, dX A_K/B_N, dW A_M/B_N, and A_M/B_K),
split-K, residual add, accumulate-into-output, and the SwiGLU forward / backward epilogues
(reference model.py:254 ``w2(silu(w1 x) * w3 x)``), on random data with asymmetric operands.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu


def K():
    from fault_tolerant_llm_training_amd._native import kernels

    return kernels()


def rnd(*s, scale=1.0):
    return ((torch.rand(*s, device="cuda") * 2 - 1) * scale).bfloat16()


def check(out, ref, K_):
    err = (out.float() - ref).abs().max().item()
    tol = 2e-2 * ref.abs().max().item() + 1e-2
    assert err <= tol, (err, tol)
    # relative Frobenius error: a wrong tile/transposition would be O(1)
    rel = ((out.float() - ref).norm() / ref.norm()).item()
    assert rel < 8e-3, rel


@pytest.fixture(params=[256, 128], ids=["tile256", "tile128"])
def tile(request):
    """Force the 256 x 256 or the 128 x 128 kernel (the default picks per shape)."""
    K().gemm_config(request.param)
    yield request.param
    K().gemm_config(0)


@pytest.mark.parametrize("a_kc,b_kc", [(True, True), (True, False), (False, False), (False, True)])
@pytest.mark.parametrize("M,N,Kd,splits", [(256, 256, 64, 1), (512, 768, 320, 1), (768, 512, 1024, 2),
                                           (512, 1024, 2048, 0), (1024, 256, 4096, 4), (384, 640, 192, 1),
                                           (128, 384, 2048, 0)])
def test_gemm_layouts(tile, a_kc, b_kc, M, N, Kd, splits):
    if M % tile or N % tile:
        pytest.skip("shape not a multiple of the tile")
    torch.manual_seed(M + N + Kd)
    A = rnd(M, Kd)
    B = rnd(Kd, N) + torch.arange(N, device="cuda").bfloat16() * 1e-3  # asymmetric
    a_arg = A.contiguous() if a_kc else A.t().contiguous()
    b_arg = B.t().contiguous() if b_kc else B.contiguous()
    out = K().gemm(a_arg, a_kc, b_arg, b_kc, M, N, Kd, None, None, False, splits)
    check(out, A.float() @ B.float(), Kd)


@pytest.mark.parametrize("splits", [1, 2])
def test_gemm_residual_and_accumulate(tile, splits):
    M, N, Kd = 512, 512, 1024
    A, B, R = rnd(M, Kd), rnd(N, Kd), rnd(M, N)
    ref = A.float() @ B.float().t()
    out = K().gemm(A, True, B, True, M, N, Kd, None, R, False, splits)
    check(out, ref + R.float(), Kd)
    C = R.clone()
    K().gemm(A, True, B, True, M, N, Kd, C, None, True, splits)
    check(C, ref + R.float(), Kd)


def test_gemm_tile_choice_gpt2_shapes():
    """Default tile choice on GPT-2-small shapes (128 tiles where 256 tiles underfill), all
    layouts, against fp32."""
    for M, N, Kd in ((2048, 768, 768), (2048, 2304, 768), (768, 768, 2048)):
        A = rnd(M, Kd)
        B = rnd(Kd, N)
        for a_kc, b_kc in ((True, True), (True, False), (False, False)):
            a_arg = A.contiguous() if a_kc else A.t().contiguous()
            b_arg = B.t().contiguous() if b_kc else B.contiguous()
            out = K().gemm(a_arg, a_kc, b_arg, b_kc, M, N, Kd, None, None, False, 0)
            check(out, A.float() @ B.float(), Kd)


def test_gemm_swiglu_forward_and_backward():
    T, D, F = 512, 512, 768
    x, w13, w2 = rnd(T, D), rnd(2 * F, D, scale=0.1), rnd(D, F, scale=0.1)
    a, gu = K().gemm_swiglu(x, w13)
    gu_ref = (x.float() @ w13.float().t())
    check(gu, gu_ref, D)
    g, u = gu.float().chunk(2, dim=-1)  # activation from the kernel's own (bf16) pre-activation
    a_ref = torch.nn.functional.silu(g) * u
    assert (a.float() - a_ref).abs().max().item() <= 1e-2 * a_ref.abs().max().item() + 1e-3
    dy = rnd(T, D)
    dgu = K().gemm_swiglu_bwd(dy, w2, gu)
    da = (dy.float() @ w2.float()).bfloat16().float()
    s = torch.sigmoid(g)
    dg_ref = da * u * (s + g * s * (1 - s))
    du_ref = da * g * s
    ref = torch.cat([dg_ref, du_ref], dim=-1)
    check(dgu, ref, D)
