"""--model-dtype fp16 / fp32 on the GPU (reference utils.py:14-19, train.py:54-59).

Every hand-written kernel in its fp16 and fp32 variants against a plain PyTorch fp32
reference; the whole tiny / gpt2-small models on the HIP path against the CPU fp32 model;
train.py end to end in fp16 / fp32 (no divergence; error -> save -> bit-exact resume).
Tolerances: fp16 keeps 11 mantissa bits (rel. ~1e-3 per rounding), fp32 is checked at ~1e-5.
"""
import math
import os

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

DTYPES = [torch.float16, torch.float32]
TOL = {torch.float16: 3e-3, torch.float32: 2e-5}


@pytest.fixture(scope="module")
def K():
    from fault_tolerant_llm_training_amd._native import kernels

    return kernels()


def rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


@pytest.mark.parametrize("dt", DTYPES)
@pytest.mark.parametrize("M,N", [(7, 768), (300, 2560), (2048, 4096), (33, 1024)])
@pytest.mark.parametrize("ln", [False, True])
def test_norm(K, dt, M, N, ln):
    torch.manual_seed(0)
    x = torch.randn(M, N, device="cuda").to(dt)
    d = torch.randn(M, N, device="cuda").to(dt)
    w = (1 + 0.1 * torch.randn(N, device="cuda")).to(dt)
    dy = torch.randn(M, N, device="cuda").to(dt)
    dres = torch.randn(M, N, device="cuda").to(dt)
    y, rstd, mean, h = K.add_norm_fwd(x, d, w, 1e-5, ln)
    assert h.dtype == dt and torch.equal(h, (x.float() + d.float()).to(dt))
    hr = h.float().requires_grad_(True)
    wr = w.float().requires_grad_(True)
    hc = hr - hr.mean(-1, keepdim=True) if ln else hr
    ref = hc * torch.rsqrt(hc.pow(2).mean(-1, keepdim=True) + 1e-5) * wr
    assert y.dtype == dt and rel(y, ref) < TOL[dt]
    dw = torch.empty_like(w)
    dx = K.norm_bwd(dy, h, w, rstd, mean if ln else None, dw, dres, False)
    gx, gw = torch.autograd.grad(ref, (hr, wr), dy.float())
    assert rel(dx, gx + dres.float()) < 2 * TOL[dt]
    assert rel(dw, gw) < 2 * TOL[dt]
    dw2 = dw.clone()
    K.norm_bwd(dy, h, w, rstd, mean if ln else None, dw2, None, True)
    assert rel(dw2, 2 * gw) < 2 * TOL[dt]


@pytest.mark.parametrize("dt", DTYPES)
def test_rope(K, dt):
    from fault_tolerant_llm_training_amd.models.llama import rope_tables
    from fault_tolerant_llm_training_amd.ops.functional import rope_reference

    B, S, hq, hkv, d = 2, 128, 8, 2, 64
    cos, sin = (t.cuda() for t in rope_tables(d, S, 10000.0))
    W = (hq + 2 * hkv) * d
    qkv = torch.randn(B * S, W, device="cuda").to(dt)
    qk = K.rope_fwd(qkv, cos, sin, S, hq, hkv, d)
    q = rope_reference(qkv[:, : hq * d].view(B, S, hq, d).float(), cos, sin).view(B * S, -1)
    k = rope_reference(qkv[:, hq * d : (hq + hkv) * d].view(B, S, hkv, d).float(), cos, sin).view(B * S, -1)
    assert qk.dtype == dt and rel(qk, torch.cat([q, k], 1)) < TOL[dt]
    g = torch.randn(B * S, W, device="cuda").to(dt)
    g2 = g.clone()
    K.rope_bwd_(g2, cos, sin, S, hq, hkv, d)
    xr = qkv.float().requires_grad_(True)
    qr = rope_reference(xr[:, : hq * d].view(B, S, hq, d), cos, sin).reshape(B * S, -1)
    kr = rope_reference(xr[:, hq * d : (hq + hkv) * d].view(B, S, hkv, d), cos, sin).reshape(B * S, -1)
    (ref,) = torch.autograd.grad(torch.cat([qr, kr, xr[:, (hq + hkv) * d :]], 1), (xr,), g.float())
    assert rel(g2, ref) < TOL[dt]


@pytest.mark.parametrize("dt", DTYPES)
def test_swiglu_xent_embedding(K, dt):
    torch.manual_seed(1)
    gu = torch.randn(300, 2 * 1408, device="cuda").to(dt)
    a = K.swiglu_fwd(gu)
    x = gu.float().requires_grad_(True)
    g_, u_ = x.chunk(2, -1)
    ref = F.silu(g_) * u_
    assert a.dtype == dt and rel(a, ref) < TOL[dt]
    da = torch.randn(300, 1408, device="cuda").to(dt)
    (gx,) = torch.autograd.grad(ref, (x,), da.float())
    assert rel(K.swiglu_bwd(da, gu), gx) < TOL[dt]

    T, V = 64, 32000
    logits = (3 * torch.randn(T, V, device="cuda")).to(dt)
    labels = torch.randint(0, V, (T,), device="cuda")
    labels[0] = -100
    loss, lse = K.xent_fwd(logits, labels, -100)
    lref = F.cross_entropy(logits.float(), labels, reduction="none", ignore_index=-100)
    assert torch.allclose(loss, lref, atol=1e-4, rtol=1e-4)
    n = (labels != -100).sum().item()
    lg = logits.clone()
    K.xent_bwd_(lg, labels, lse, torch.tensor([1.0], device="cuda"), torch.tensor([1.0 / n], device="cuda"), -100)
    xl = logits.float().requires_grad_(True)
    (gl,) = torch.autograd.grad(F.cross_entropy(xl, labels, reduction="sum", ignore_index=-100) / n, (xl,))
    assert rel(lg, gl) < TOL[dt]

    Vv, D, Tt = 1000, 256, 512
    w = torch.randn(Vv, D, device="cuda").to(dt)
    tok = torch.randint(0, 50, (Tt,), device="cuda")
    assert torch.equal(K.embedding_fwd(tok, w), w[tok])
    dy = torch.randn(Tt, D, device="cuda").to(dt)
    dw = torch.zeros(Vv, D, device="cuda").to(dt)
    K.embedding_bwd_(dy, tok, dw, False)
    ref = torch.zeros(Vv, D, device="cuda").index_add_(0, tok, dy.float())
    assert rel(dw, ref) < TOL[dt]


@pytest.mark.parametrize("pdt,sdt", [(torch.float16, torch.float16), (torch.float16, torch.float32),
                                     (torch.float32, torch.float32)])
def test_grad_norm_adamw(K, pdt, sdt):
    from fault_tolerant_llm_training_amd.optim.adamw import _adamw_reference

    n = 1 << 20
    g = (0.01 * torch.randn(n, device="cuda")).to(pdt)
    p = torch.randn(n, device="cuda").to(pdt)
    m = (0.001 * torch.randn(n, device="cuda")).to(sdt)
    v = (1e-5 * torch.rand(n, device="cuda")).to(sdt)
    stats = torch.zeros(3, device="cuda")
    K.grad_norm_(g, stats, 1.0)
    ref_norm = g.double().norm().item()
    assert math.isclose(stats[0].item(), ref_norm, rel_tol=1e-5)
    p1, m1, v1 = p.clone(), m.clone(), v.clone()
    K.adamw_(p1, g, m1, v1, stats, 1e-3, 0.9, 0.999, 1e-8, 0.01, 3)
    p2, m2, v2 = p.clone(), m.clone(), v.clone()
    _adamw_reference(p2, g, m2, v2, stats, 1e-3, 0.9, 0.999, 1e-8, 0.01, 3)
    # same fp32 math, same rounding to the storage dtype: agreement up to one ulp of fp32 ops
    assert rel(p1, p2) < 1e-5 and rel(m1, m2) < 1e-5 and rel(v1, v2) < 1e-5


def ref_attn(q, k, v):
    B, S, Hq, D = q.shape
    rep = Hq // k.shape[2]
    k = k.repeat_interleave(rep, 2)
    v = v.repeat_interleave(rep, 2)
    s = torch.einsum("bqhd,bkhd->bhqk", q, k) / D**0.5
    s = s.masked_fill(torch.ones(S, S, dtype=torch.bool, device=q.device).triu(1), float("-inf"))
    return torch.einsum("bhqk,bkhd->bqhd", s.softmax(-1), v)


@pytest.mark.parametrize("dt", DTYPES)
@pytest.mark.parametrize("B,S,Hq,Hkv,D", [(1, 256, 4, 2, 128), (2, 192, 4, 4, 64), (1, 1000, 8, 2, 64),
                                          (1, 2048, 12, 12, 64), (3, 100, 4, 1, 128)])
def test_flash(dt, B, S, Hq, Hkv, D):
    from fault_tolerant_llm_training_amd.ops.attention import flash_attn_bwd, flash_attn_fwd

    torch.manual_seed(0)
    T = B * S
    qkv = torch.randn(T, (Hq + 2 * Hkv) * D, device="cuda").to(dt)
    qk = torch.randn(T, (Hq + Hkv) * D, device="cuda").to(dt)
    o, lse = flash_attn_fwd(qk, qkv, S, Hq, Hkv, D)
    q = qk[:, : Hq * D].double().view(B, S, Hq, D).requires_grad_(True)
    k = qk[:, Hq * D :].double().view(B, S, Hkv, D).requires_grad_(True)
    v = qkv[:, (Hq + Hkv) * D :].double().view(B, S, Hkv, D).requires_grad_(True)
    ref = ref_attn(q, k, v)
    assert o.dtype == dt and rel(o.view(B, S, Hq, D), ref) < TOL[dt]
    do = torch.randn(T, Hq * D, device="cuda").to(dt)
    dqkv = flash_attn_bwd(do, qk, qkv, o, lse, S, Hq, Hkv, D)
    gq, gk, gv = torch.autograd.grad(ref, (q, k, v), do.double().view(B, S, Hq, D))
    tol = 3 * TOL[dt]  # fp16: dS / P rounded to fp16 for the MFMAs
    assert rel(dqkv[:, : Hq * D].view(B, S, Hq, D), gq) < tol
    assert rel(dqkv[:, Hq * D : (Hq + Hkv) * D].view(B, S, Hkv, D), gk) < tol
    assert rel(dqkv[:, (Hq + Hkv) * D :].view(B, S, Hkv, D), gv) < tol
    again = flash_attn_bwd(do, qk, qkv, o, lse, S, Hq, Hkv, D)
    assert torch.equal(dqkv, again)  # deterministic backward in every dtype


@pytest.mark.parametrize("M,N,Kd", [(2048, 6144, 4096), (512, 1024, 256), (256, 3072, 768)])
def test_gemm_w4_fp16(K, M, N, Kd):
    torch.manual_seed(0)
    a = torch.randn(M, Kd, device="cuda").half()
    b = torch.randn(N, Kd, device="cuda").half()
    r = torch.randn(M, N, device="cuda").half()
    for nj in (8, 6, 4):
        if N % (32 * nj):
            continue
        ref = a.float() @ b.float().t()
        assert rel(K.gemm_nt_w4(a, b, None, None, nj), ref) < 2e-3
        assert rel(K.gemm_nt_w4(a, b, None, r, nj), ref + r.float()) < 2e-3


def test_gemm_qkv_rope_w4_fp16(K):
    from fault_tolerant_llm_training_amd.models.llama import rope_tables

    S, hq, hkv, d, Kd = 512, 16, 4, 64, 1024
    cos, sin = (t.cuda() for t in rope_tables(d, S, 10000.0))
    x = torch.randn(2 * S, Kd, device="cuda").half()
    w = (torch.randn((hq + 2 * hkv) * d, Kd, device="cuda") / 32).half()
    out = K.gemm_qkv_rope_w4(x, w, cos, sin, S, hq, hkv, d)
    ref = K.gemm_nt_w4(x, w, None, None, 0)
    K.rope_bwd_(out, cos, sin, S, hq, hkv, d)  # rotate back: the unrotated projection
    assert rel(out, ref) < 3e-3


@pytest.mark.parametrize("dt", DTYPES)
@pytest.mark.parametrize("preset,V,S", [("tiny", 512, 128), ("gpt2-small", 1024, 256)])
def test_model_gpu_vs_cpu(dt, preset, V, S):
    """The whole model in ``dt`` on the HIP path vs the fp32 CPU model with the same weights."""
    from fault_tolerant_llm_training_amd.models.llama import build_model, model_args_for

    a = model_args_for(preset, vocab_size=V, seq_len=S)
    mg = build_model(a, "cuda", dt, seed=7)
    mc = build_model(a, "cpu", torch.float32, seed=7)
    mc.load_state_dict({k: v.float().cpu() for k, v in mg.state_dict().items()})
    torch.manual_seed(3)
    tok = torch.randint(0, V, (2, S))
    lab = torch.randint(0, V, (2, S))
    lg = mg(tok.cuda(), lab.cuda())
    lc = mc(tok, lab)
    lg.backward()
    lc.backward()
    assert mg.flat.grads.dtype == dt
    assert abs(lg.item() - lc.item()) < (2e-3 if dt == torch.float16 else 2e-5) * abs(lc.item())
    assert rel(mg.flat.grads.cpu(), mc.flat.grads) < (2e-2 if dt == torch.float16 else 1e-4)


def test_model_gpu_fp64_vs_cpu():
    """--model-dtype fp64 on the GPU (no HIP kernel covers fp64: composed PyTorch ops on the device)
    == the fp64 CPU model with the same weights (the cross-entropy runs in fp32 on both, as in the
    reference's logits.float(): agreement to fp32 rounding)."""
    from fault_tolerant_llm_training_amd.models.llama import build_model, model_args_for

    a = model_args_for("tiny", vocab_size=512, seq_len=128)
    mg = build_model(a, "cuda", torch.float64, seed=7)
    mc = build_model(a, "cpu", torch.float64, seed=7)
    mc.load_state_dict({k: v.cpu() for k, v in mg.state_dict().items()})
    torch.manual_seed(3)
    tok = torch.randint(0, 512, (2, 128))
    lab = torch.randint(0, 512, (2, 128))
    lg = mg(tok.cuda(), lab.cuda())
    lc = mc(tok, lab)
    lg.backward()
    lc.backward()
    assert mg.flat.grads.dtype == torch.float64 and mg.flat.grads.is_cuda
    assert abs(lg.item() - lc.item()) < 1e-6 * abs(lc.item())
    assert rel(mg.flat.grads.cpu(), mc.flat.grads) < 1e-5


GPU = ["--device", "cuda", "--synthetic-data", "--vocab-size", "1024", "--sequence-length", "256",
       "--batch-size", "2", "--learning-rate", "1e-3", "--lr-warmup-steps", "3", "--logging-frequency", "5"]


@pytest.mark.parametrize("dt", ["fp16", "fp32", "fp64"])
def test_train_error_save_resume_bit_exact(tmp_path, dt):
    """train.py --model-dtype fp16 / fp32 / fp64 on the GPU (fp64: the composed-PyTorch path, as the
    reference allows, utils.py:14-19): an injected error saves, the resumed job ends bit-identical
    to an uninterrupted one, and the losses stay finite and bounded."""
    from helpers import run_train, write_fake_sbatch

    d = str(tmp_path)
    write_fake_sbatch(d)
    base = GPU + ["--model", "tiny", "--model-dtype", dt, "--checkpoint-path", os.path.join(d, "ck"),
                  "--training-steps", "31"]
    rc, out = run_train(d, "800", base + ["--raise-error", "--error-step", "30"], timeout=240)
    assert rc == 0 and "Checkpoint saved at step 30" in out, out[-3000:]
    losses = [float(l.split("Loss: ")[1].split()[0].rstrip("|,")) for l in out.splitlines() if "Loss: " in l]
    # uniform synthetic tokens: the loss stays near ln(V) = 6.93 (no divergence)
    assert len(losses) >= 3 and all(math.isfinite(x) and x < math.log(1024) + 0.5 for x in losses), losses
    rc, out = run_train(d, "801", base + ["--raise-error", "--error-step", "12"], timeout=240)
    assert rc == 0 and "Checkpoint saved at step 12" in out, out[-3000:]
    rc, out = run_train(d, "802", base + ["--raise-error", "--error-step", "30", "--checkpoint-id", "801"],
                        timeout=240)
    assert rc == 0 and "Resuming training from training_step 12" in out, out[-3000:]
    ld = lambda j: torch.load(os.path.join(d, "ck", f"checkpoint_{j}.ckpt"), map_location="cpu",
                              weights_only=True)
    a, c = ld(800), ld(802)
    want = {"fp16": torch.float16, "fp32": torch.float32, "fp64": torch.float64}[dt]
    for k in a["model"]:
        assert a["model"][k].dtype == want
        assert torch.equal(a["model"][k], c["model"][k]), k
    for i in a["optimizer"]["state"]:
        assert torch.equal(a["optimizer"]["state"][i]["exp_avg"], c["optimizer"]["state"][i]["exp_avg"])
        assert torch.equal(a["optimizer"]["state"][i]["exp_avg_sq"], c["optimizer"]["state"][i]["exp_avg_sq"])


@pytest.mark.parametrize("dt", ["fp16", "fp32"])
def test_train_gpt2_small(tmp_path, dt):
    """gpt2-small trains in fp16 / fp32 on the GPU (finite, bounded losses over 20 steps)."""
    from helpers import run_train, write_fake_sbatch

    d = str(tmp_path)
    write_fake_sbatch(d)
    rc, out = run_train(d, "810", GPU + ["--model", "gpt2-small", "--model-dtype", dt, "--training-steps", "20"],
                        timeout=300)
    assert rc == 0, out[-3000:]
    losses = [float(l.split("Loss: ")[1].split()[0].rstrip("|,")) for l in out.splitlines() if "Loss: " in l]
    # uniform synthetic tokens: the loss stays near ln(V) = 6.93 (no divergence)
    assert len(losses) >= 3 and all(math.isfinite(x) and x < math.log(1024) + 0.5 for x in losses), losses
