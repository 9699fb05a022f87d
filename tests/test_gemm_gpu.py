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


@pytest.mark.parametrize("nj", [8, 7, 6, 4])
@pytest.mark.parametrize("M,K", [(256, 128), (512, 256), (2048, 4096), (768, 768)])
def test_gemm_w4_tiles(nj, M, K):
    """4-wave schedule-level GEMM (csrc/kernels/gemm_w4.hip), every tile width, vs fp32; residual."""
    from fault_tolerant_llm_training_amd._native import kernels

    K_ = kernels()
    N = 32 * nj * 3
    torch.manual_seed(M + K + nj)
    a = (torch.rand(M, K, device="cuda") * 2 - 1).bfloat16()
    b = (torch.rand(N, K, device="cuda") * 2 - 1).bfloat16()
    ref = a.float() @ b.float().t()
    out = K_.gemm_nt_w4(a, b, None, None, nj)
    assert ((out.float() - ref).norm() / ref.norm()).item() < 4e-3
    r = (torch.rand(M, N, device="cuda") * 2 - 1).bfloat16()
    out = K_.gemm_nt_w4(a, b, None, r, nj)
    ref = ref + r.float()
    assert ((out.float() - ref).norm() / ref.norm()).item() < 4e-3
    o2 = torch.empty_like(out)
    K_.gemm_nt_w4(a, b, o2, r, nj)
    assert torch.equal(o2, out)  # deterministic


@pytest.mark.parametrize("hq,hkv,d,S,B", [(32, 8, 128, 2048, 1), (12, 12, 64, 512, 2), (16, 4, 64, 256, 4)])
def test_gemm_qkv_rope_w4(hq, hkv, d, S, B):
    """QKV projection with RoPE in the epilogue == projection (fp32) then the reference RoPE."""
    from fault_tolerant_llm_training_amd._native import kernels
    from fault_tolerant_llm_training_amd.models.llama import rope_tables
    from fault_tolerant_llm_training_amd.ops.functional import rope_reference

    K_ = kernels()
    D = 1024 if hq * d <= 1024 else 4096
    W = (hq + 2 * hkv) * d
    torch.manual_seed(hq)
    x = (torch.rand(B * S, D, device="cuda") * 2 - 1).bfloat16()
    w = ((torch.rand(W, D, device="cuda") * 2 - 1) / D ** 0.5).bfloat16()
    cos, sin = rope_tables(d, S, 500000.0)
    cos, sin = cos.cuda(), sin.cuda()
    if K_.gemm_w4_pick(B * S, W) == 0:
        pytest.skip("no w4 tile width for this N")
    out = K_.gemm_qkv_rope_w4(x, w, cos, sin, S, hq, hkv, d)
    y = (x.float() @ w.float().t()).bfloat16()  # the unfused path rotates the bf16 projection
    q = rope_reference(y[:, : hq * d].view(B, S, hq, d), cos, sin).reshape(B * S, -1)
    k = rope_reference(y[:, hq * d : (hq + hkv) * d].view(B, S, hkv, d), cos, sin).reshape(B * S, -1)
    ref = torch.cat([q, k, y[:, (hq + hkv) * d :]], 1).float()
    assert ((out.float() - ref).norm() / ref.norm()).item() < 6e-3


@pytest.mark.parametrize("T,N,Kd", [(2048, 6144, 4096), (512, 1024, 768)])
def test_weight_grad_on_w4(T, N, Kd):
    """dW = dY^T X through the 4-wave kernel (transposed operands) into a gradient sink, written
    and accumulated (gradient accumulation), vs fp32."""
    from fault_tolerant_llm_training_amd.ops import functional as Fx
    from fault_tolerant_llm_training_amd.ops.grad_sink import GradSink

    torch.manual_seed(T + N)
    dy = rnd(T, N)
    x = rnd(T, Kd)
    buf = torch.zeros(N * Kd, device="cuda", dtype=torch.bfloat16)
    sink = GradSink(buf, 0, N * Kd)
    old = Fx._W4_DW
    Fx.set_w4_dw(True)
    try:
        Fx.weight_grad(dy, x, sink)
        ref = dy.float().t() @ x.float()
        assert ((buf.view(N, Kd).float() - ref).norm() / ref.norm()).item() < 4e-3
        sink.accumulate = True
        Fx.weight_grad(dy, x, sink)
        assert ((buf.view(N, Kd).float() - 2 * ref).norm() / (2 * ref).norm()).item() < 6e-3
    finally:
        Fx.set_w4_dw(old)


@pytest.mark.parametrize("ks", [0, 1, 2, 4])
@pytest.mark.parametrize("M,N,K", [(128, 128, 64), (2048, 768, 768), (2048, 2304, 768), (2048, 768, 2048),
                                   (256, 384, 4096), (2048, 1024, 2816)])
def test_gemm_s_tiles(M, N, K, ks):
    """128 x 128-tile GEMM (csrc/kernels/gemm_s.hip) incl. split-K, vs fp32; residual; bitwise
    reproducible (the split-K slices are summed in a fixed order by the last-arriving workgroup)."""
    from fault_tolerant_llm_training_amd._native import kernels

    K_ = kernels()
    torch.manual_seed(M + N + K + ks)
    a = (torch.rand(M, K, device="cuda") * 2 - 1).bfloat16()
    b = (torch.rand(N, K, device="cuda") * 2 - 1).bfloat16()
    ref = a.float() @ b.float().t()
    out = K_.gemm_nt_s(a, b, None, None, ks)
    assert ((out.float() - ref).norm() / ref.norm()).item() < 4e-3
    r = (torch.rand(M, N, device="cuda") * 2 - 1).bfloat16()
    out = K_.gemm_nt_s(a, b, None, r, ks)
    ref = ref + r.float()
    assert ((out.float() - ref).norm() / ref.norm()).item() < 4e-3
    for _ in range(3):
        o2 = torch.empty_like(out)
        K_.gemm_nt_s(a, b, o2, r, ks)
        assert torch.equal(o2, out)


def test_gemm_s_fp16():
    from fault_tolerant_llm_training_amd._native import kernels

    K_ = kernels()
    torch.manual_seed(7)
    a = (torch.rand(512, 768, device="cuda") * 2 - 1).half()
    b = (torch.rand(384, 768, device="cuda") * 2 - 1).half()
    ref = a.float() @ b.float().t()
    out = K_.gemm_nt_s(a, b, None, None, 0)
    assert out.dtype == torch.float16
    assert ((out.float() - ref).norm() / ref.norm()).item() < 2e-3


@pytest.mark.parametrize("M,F,K", [(256, 448, 128), (512, 1792, 768), (2048, 14336, 4096)])
def test_gemm_swiglu_w4(M, F, K):
    """w1|w3 GEMM with SwiGLU in the epilogue: gu equals the plain w4 GEMM bitwise (same MFMA order),
    a / a^T equal swiglu_fwd_t of that gu bitwise, and all match fp32 (reference model.py:254)."""
    from fault_tolerant_llm_training_amd._native import kernels

    K_ = kernels()
    torch.manual_seed(M + F + K)
    x = (torch.rand(M, K, device="cuda") * 2 - 1).bfloat16()
    w13 = ((torch.rand(2 * F, K, device="cuda") * 2 - 1) * (1.0 / K**0.5)).bfloat16()
    gu, a, aT = K_.gemm_swiglu_w4(x, w13)
    assert torch.equal(gu, K_.gemm_nt_w4(x, w13, None, None, 7))
    a2, aT2 = K_.swiglu_fwd_t(gu, True)
    assert torch.equal(a, a2) and torch.equal(aT, aT2)
    ref = x.float() @ w13.float().t()
    g, u = ref[:, :F], ref[:, F:]
    aref = torch.nn.functional.silu(g) * u
    assert ((gu.float() - ref).norm() / ref.norm()).item() < 4e-3
    assert ((a.float() - aref).norm() / aref.norm()).item() < 1e-2
