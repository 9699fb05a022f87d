"""Hand-written gfx950 GEMMs vs an fp32 PyTorch reference: the w4 kernel's forward layout with the
residual, RoPE (reference model.py:100-126, 195) and SwiGLU (model.py:254) epilogues, the weight
gradient through the routing into a gradient sink, and the 128 x 128-tile kernel (gemm_s.hip).
The k-major (dX / dW) layouts and split-K: tests/test_gemm_w4t_gpu.py.
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
def test_weight_grad_on_w4(T, N, Kd, monkeypatch):
    """dW = dY^T X through the routing onto the w4 kernel (k-major operands as stored) into a
    gradient sink, written and accumulated (gradient accumulation), vs fp32."""
    from fault_tolerant_llm_training_amd.ops import functional as Fx
    from fault_tolerant_llm_training_amd.ops.grad_sink import GradSink

    monkeypatch.setattr(Fx, "_W4_MIN_TILES", 1)

    monkeypatch.setattr(Fx, "_W4_DEEP_K", 0)
    torch.manual_seed(T + N)
    dy = rnd(T, N)
    x = rnd(T, Kd)
    assert Fx._w4_dw_ok(T, N, Kd, dy, x)
    buf = torch.zeros(N * Kd, device="cuda", dtype=torch.bfloat16)
    sink = GradSink(buf, 0, N * Kd)
    Fx.weight_grad(dy, x, sink)
    ref = dy.float().t() @ x.float()
    assert ((buf.view(N, Kd).float() - ref).norm() / ref.norm()).item() < 4e-3
    sink.accumulate = True
    Fx.weight_grad(dy, x, sink)
    assert ((buf.view(N, Kd).float() - 2 * ref).norm() / (2 * ref).norm()).item() < 6e-3


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


@pytest.mark.parametrize("M,F,K", [(256, 448, 128), (512, 1792, 768), (2048, 14336, 4096), (2048, 2048, 768),
                                   (2048, 2816, 1024)])
def test_gemm_swiglu_w4(M, F, K):
    """w1|w3 GEMM with SwiGLU in the epilogue: gu equals the plain w4 GEMM bitwise (same MFMA order),
    a equals the SwiGLU kernel on that gu bitwise and a^T its transpose, and all match fp32
    (reference model.py:254)."""
    from fault_tolerant_llm_training_amd._native import kernels

    K_ = kernels()
    torch.manual_seed(M + F + K)
    x = (torch.rand(M, K, device="cuda") * 2 - 1).bfloat16()
    w13 = ((torch.rand(2 * F, K, device="cuda") * 2 - 1) * (1.0 / K**0.5)).bfloat16()
    gu, a, aT = K_.gemm_swiglu_w4(x, w13)
    nj = K_.gemm_swiglu_pick(M, F)  # 7 for the 8B F = 14336; 4 / 8 for GPT-2's 2048 / 2816
    assert torch.equal(gu, K_.gemm_nt_w4(x, w13, None, None, nj))
    assert torch.equal(a, K_.swiglu_fwd(gu)) and torch.equal(aT, a.t().contiguous())
    ref = x.float() @ w13.float().t()
    g, u = ref[:, :F], ref[:, F:]
    aref = torch.nn.functional.silu(g) * u
    assert ((gu.float() - ref).norm() / ref.norm()).item() < 4e-3
    assert ((a.float() - aref).norm() / aref.norm()).item() < 1e-2
