"""Numerics of every hand-written HIP kernel vs a plain PyTorch fp32 reference."""
import math

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def K():
    from fault_tolerant_llm_training_amd._native import kernels

    return kernels()


def rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


@pytest.mark.parametrize("M,N", [(1, 128), (7, 768), (2048, 4096), (33, 1024), (5, 8192), (300, 2560), (4099, 2048)])
@pytest.mark.parametrize("ln", [False, True])
def test_norm(K, M, N, ln):
    torch.manual_seed(0)
    x = torch.randn(M, N, device="cuda").bfloat16()
    w = (1 + 0.1 * torch.randn(N, device="cuda")).bfloat16()
    dy = torch.randn(M, N, device="cuda").bfloat16()
    y, rstd, mean = K.norm_fwd(x, w, 1e-5, ln)
    xr = x.float().requires_grad_(True)
    wr = w.float().requires_grad_(True)
    xc = xr - xr.mean(-1, keepdim=True) if ln else xr
    ref = xc * torch.rsqrt(xc.pow(2).mean(-1, keepdim=True) + 1e-5) * wr
    assert rel(y, ref) < 1e-2
    dw = torch.empty_like(w)
    dx = K.norm_bwd(dy, x, w, rstd, mean if ln else None, dw, None, False)
    gx, gw = torch.autograd.grad(ref, (xr, wr), dy.float())
    assert rel(dx, gx) < 2e-2
    assert rel(dw, gw) < 2e-2


@pytest.mark.parametrize("B,S,hq,hkv,d", [(1, 64, 4, 2, 128), (2, 128, 8, 8, 64), (1, 2048, 32, 8, 128)])
def test_rope(K, B, S, hq, hkv, d):
    from fault_tolerant_llm_training_amd.models.llama import rope_tables
    from fault_tolerant_llm_training_amd.ops.functional import rope_reference

    cos, sin = rope_tables(d, S, 500000.0)
    cos, sin = cos.cuda(), sin.cuda()
    W = (hq + 2 * hkv) * d
    qkv = torch.randn(B * S, W, device="cuda").bfloat16()
    qk = K.rope_fwd(qkv, cos, sin, S, hq, hkv, d)
    q = rope_reference(qkv[:, : hq * d].view(B, S, hq, d).float(), cos, sin).view(B * S, -1)
    k = rope_reference(qkv[:, hq * d : (hq + hkv) * d].view(B, S, hkv, d).float(), cos, sin).view(B * S, -1)
    assert rel(qk, torch.cat([q, k], 1)) < 1e-2
    # backward is the transpose rotation: <R x, y> == <x, R^T y>
    dq = torch.randn(B * S, W, device="cuda").bfloat16()
    d2 = dq.clone()
    K.rope_bwd_(d2, cos, sin, S, hq, hkv, d)
    xr = qkv.float().requires_grad_(True)
    qr = rope_reference(xr[:, : hq * d].view(B, S, hq, d), cos, sin).reshape(B * S, -1)
    kr = rope_reference(xr[:, hq * d : (hq + hkv) * d].view(B, S, hkv, d), cos, sin).reshape(B * S, -1)
    out = torch.cat([qr, kr, xr[:, (hq + hkv) * d :]], 1)
    (g,) = torch.autograd.grad(out, (xr,), dq.float())
    assert rel(d2, g) < 1e-2


@pytest.mark.parametrize("T,F_", [(1, 64), (300, 1408), (2048, 14336)])
def test_swiglu(K, T, F_):
    gu = torch.randn(T, 2 * F_, device="cuda").bfloat16()
    a = K.swiglu_fwd(gu)
    x = gu.float().requires_grad_(True)
    g, u = x.chunk(2, -1)
    ref = F.silu(g) * u
    assert rel(a, ref) < 1e-2
    da = torch.randn(T, F_, device="cuda").bfloat16()
    dgu = K.swiglu_bwd(da, gu)
    (gx,) = torch.autograd.grad(ref, (x,), da.float())
    assert rel(dgu, gx) < 1e-2


@pytest.mark.parametrize("T,V", [(3, 1024), (64, 32000), (16, 131072), (70000, 64)])
def test_xent(K, T, V):
    logits = (3 * torch.randn(T, V, device="cuda")).bfloat16()
    labels = torch.randint(0, V, (T,), device="cuda")
    labels[0] = -100
    loss, lse = K.xent_fwd(logits, labels, -100)
    ref = F.cross_entropy(logits.float(), labels, reduction="none", ignore_index=-100)
    assert torch.allclose(loss, ref, atol=2e-3, rtol=1e-3)
    n = (labels != -100).sum().item()
    inv = torch.tensor([1.0 / n], device="cuda")
    g = torch.tensor([2.0], device="cuda")
    lg = logits.clone()
    K.xent_bwd_(lg, labels, lse, g, inv, -100)
    x = logits.float().requires_grad_(True)
    l2 = F.cross_entropy(x, labels, reduction="sum", ignore_index=-100) / n * 2.0
    (gx,) = torch.autograd.grad(l2, (x,))
    assert rel(lg, gx) < 1e-2


@pytest.mark.parametrize("V,T,ntok", [(1000, 512, 50), (131072, 2048, 131072), (131072, 16384, 3000),
                                      (70000, 20001, 7), (64, 1, 64), (131072, 4096, 1)])
def test_embedding(K, V, T, ntok):
    """Forward gather; backward = in-tree stable radix sort + per-token fp32 segment sums in row
    order. Compared bit-exactly with the same sums formed in that order on the CPU."""
    D = 256
    torch.manual_seed(T)
    w = torch.randn(V, D, device="cuda").bfloat16()
    tok = torch.randint(0, ntok, (T,), device="cuda")  # ntok << T: many duplicates
    out = K.embedding_fwd(tok, w)
    assert torch.equal(out, w[tok])
    dy = torch.randn(T, D, device="cuda").bfloat16()
    dw = torch.full((V, D), 7.0, device="cuda").bfloat16()
    K.embedding_bwd_(dy, tok, dw, False)
    # reference: each token's rows added in ascending row order (occurrence rank by rank)
    t = tok.cpu()
    order = torch.sort(t, stable=True).indices
    st = t[order]
    first = torch.ones_like(st, dtype=torch.bool)
    first[1:] = st[1:] != st[:-1]
    seg_start = torch.cummax(torch.where(first, torch.arange(T), torch.zeros(T, dtype=torch.long)), 0).values
    occ = torch.arange(T) - seg_start
    acc = torch.zeros(V, D)
    dyc = dy.cpu().float()
    for r in range(int(occ.max()) + 1):
        sel = order[occ == r]
        acc.index_add_(0, t[sel], dyc[sel])
    assert torch.equal(dw.cpu(), acc.bfloat16())
    dw2 = dw.clone()
    K.embedding_bwd_(dy, tok, dw2, True)  # accumulate into the existing rows
    assert rel(dw2.cpu(), 2 * acc) < 1e-2


@pytest.mark.parametrize("state_dtype", [torch.bfloat16, torch.float32])
def test_grad_norm_adamw(K, state_dtype):
    from fault_tolerant_llm_training_amd.optim.adamw import _adamw_reference

    n = 1 << 20
    g = torch.randn(n, device="cuda").bfloat16()
    p = torch.randn(n, device="cuda").bfloat16()
    m = (0.1 * torch.randn(n, device="cuda")).to(state_dtype)
    v = (0.01 * torch.rand(n, device="cuda")).to(state_dtype)
    stats = torch.zeros(3, device="cuda")
    K.grad_norm_(g, stats, 1.0)
    ref_norm = g.float().norm().item()
    assert math.isclose(stats[0].item(), ref_norm, rel_tol=1e-4)
    assert math.isclose(stats[1].item(), 1.0 / (ref_norm + 1e-6), rel_tol=1e-4)
    p1, m1, v1 = p.clone(), m.clone(), v.clone()
    K.adamw_(p1, g, m1, v1, stats, 1e-3, 0.9, 0.999, 1e-8, 0.01, 3)
    p2, m2, v2 = p.clone(), m.clone(), v.clone()
    _adamw_reference(p2, g, m2, v2, stats, 1e-3, 0.9, 0.999, 1e-8, 0.01, 3)
    assert rel(p1, p2) < 1e-3 and rel(m1, m2) < 1e-2 and rel(v1, v2) < 1e-2
    # non-finite gradients skip the update
    g[5] = float("inf")
    K.grad_norm_(g, stats, 1.0)
    assert stats[2].item() == 1.0
    p3 = p.clone()
    K.adamw_(p3, g, m.clone(), v.clone(), stats, 1e-3, 0.9, 0.999, 1e-8, 0.01, 3)
    assert torch.equal(p3, p)


def test_tiny_model_gpu_vs_cpu():
    """Whole model on the HIP path vs the CPU reference path: loss and all grads."""
    from fault_tolerant_llm_training_amd.models.llama import build_model, model_args_for

    a = model_args_for("tiny", vocab_size=512, seq_len=64)
    mg = build_model(a, "cuda", torch.bfloat16, seed=7)
    mc = build_model(a, "cpu", torch.bfloat16, seed=7)
    mc.load_state_dict({k: v.cpu() for k, v in mg.state_dict().items()})
    tok = torch.randint(0, 512, (2, 64))
    lab = torch.randint(0, 512, (2, 64))
    lg = mg(tok.cuda(), lab.cuda())
    lc = mc(tok, lab)
    lg.backward()
    lc.backward()
    assert abs(lg.item() - lc.item()) < 2e-2
    assert rel(mg.flat.grads.cpu(), mc.flat.grads) < 3e-2


@pytest.mark.parametrize("max_norm", [0.0, 1e-3])
def test_pipelined_optimizer_matches_serial(max_norm):
    """Side-stream sumsq + per-bucket AdamW gated into the next forward == one serial AdamW pass."""
    from fault_tolerant_llm_training_amd.models.llama import build_model, model_args_for
    from fault_tolerant_llm_training_amd.optim.adamw import FlatAdamW
    from fault_tolerant_llm_training_amd.parallel.ddp import GradReducer

    a = model_args_for("tiny", vocab_size=512, seq_len=64)
    tok = torch.randint(0, 512, (2, 64), device="cuda")
    lab = torch.randint(0, 512, (2, 64), device="cuda")
    out = []
    for pipelined in (False, True):
        m = build_model(a, "cuda", torch.bfloat16, seed=11)
        red = GradReducer(m.flat, m.sinks_in_backward_order(), bucket_mb=0.25) if pipelined else None
        opt = FlatAdamW(m.parameters(), m.flat, lr=1e-2, max_grad_norm=max_norm, reducer=red)
        m.gate = opt.gate
        losses = []
        for _ in range(3):
            loss = m(tok, lab)
            loss.backward()
            if red is not None:
                red.finish()
            opt.step()
            losses.append(loss.float())
        opt.gate.wait_all()
        torch.cuda.synchronize()
        if pipelined:
            assert len(red.buckets) > 3
        out.append((m.flat.params.clone(), torch.stack(losses), opt.stats.clone()))
    (p0, l0, s0), (p1, l1, s1) = out
    if max_norm == 0.0:
        assert torch.allclose(s0[0], s1[0], rtol=1e-5)
        assert torch.equal(p0, p1) and torch.equal(l0, l1)
    else:  # the norm's partial-sum split differs -> clip coefficient differs in the last bits
        assert rel(p0, p1) < 1e-2 and rel(s0[:1], s1[:1]) < 1e-2


def test_activation_checkpointing_bitwise():
    """Recomputed blocks (pipelined optimizer, dW stream, bucketed reducer) train bit-identically."""
    from fault_tolerant_llm_training_amd.models.llama import build_model, model_args_for
    from fault_tolerant_llm_training_amd.optim.adamw import FlatAdamW
    from fault_tolerant_llm_training_amd.parallel.ddp import GradReducer

    a = model_args_for("tiny", vocab_size=512, seq_len=128)
    tok = torch.randint(0, 512, (2, 128), device="cuda")
    lab = torch.randint(0, 512, (2, 128), device="cuda")
    out = []
    for n, recompute_attention in ((0, False), (-1, False), (-1, True)):
        m = build_model(a, "cuda", torch.bfloat16, seed=11)
        m.set_activation_checkpointing(n, recompute_attention=recompute_attention)
        red = GradReducer(m.flat, m.sinks_in_backward_order(), bucket_mb=0.25)
        opt = FlatAdamW(m.parameters(), m.flat, lr=1e-2, max_grad_norm=1.0, reducer=red)
        m.gate = opt.gate
        losses = []
        for _ in range(3):
            loss = m(tok, lab)
            loss.backward()
            red.finish()
            opt.step()
            losses.append(loss.float())
        opt.gate.wait_all()
        torch.cuda.synchronize()
        out.append((m.flat.params.clone(), opt.exp_avg.clone(), torch.stack(losses)))
    for other in out[1:]:
        for x, y in zip(out[0], other):
            assert torch.equal(x, y)


@pytest.mark.parametrize("w4", [False, True])
def test_dw_side_stream_bitwise(w4, monkeypatch):
    """Weight-gradient GEMMs on the side stream (concurrent with dX) give bit-identical training,
    for the hipBLASLt dW (side stream) and the w4 dW (inline by default, forced onto the side
    stream here)."""
    from fault_tolerant_llm_training_amd.models.llama import build_model, model_args_for
    from fault_tolerant_llm_training_amd.ops import functional as Fx
    from fault_tolerant_llm_training_amd.optim.adamw import FlatAdamW
    from fault_tolerant_llm_training_amd.parallel.ddp import GradReducer

    if w4:
        monkeypatch.setattr(Fx, "_W4_MIN_TILES", 1)
        monkeypatch.setattr(Fx, "_W4_DEEP_K", 0)
        monkeypatch.setattr(Fx, "_W4_DW_SIDE", True)
    a = model_args_for("tiny", vocab_size=1024, seq_len=256)
    tok = torch.randint(0, 1024, (2, 256), device="cuda")
    lab = torch.randint(0, 1024, (2, 256), device="cuda")
    out = []
    try:
        for side in (False, True):
            Fx.set_dw_stream(side)
            m = build_model(a, "cuda", torch.bfloat16, seed=5)
            red = GradReducer(m.flat, m.sinks_in_backward_order(), bucket_mb=0.25)
            opt = FlatAdamW(m.parameters(), m.flat, lr=1e-2, max_grad_norm=1.0, reducer=red)
            m.gate = opt.gate
            losses = []
            for _ in range(3):
                loss = m(tok, lab)
                loss.backward()
                red.finish()
                opt.step()
                losses.append(loss.float())
            opt.gate.wait_all()
            torch.cuda.synchronize()
            out.append((m.flat.params.clone(), m.flat.grads.clone(), torch.stack(losses)))
    finally:
        Fx.set_dw_stream(True)
    (p0, g0, l0), (p1, g1, l1) = out
    assert torch.equal(g0, g1) and torch.equal(p0, p1) and torch.equal(l0, l1)


def test_weight_grad_blas_route():
    """A dW too small for the w4 kernel goes to hipBLASLt (dy^T x on the stored layouts) vs fp32."""
    from fault_tolerant_llm_training_amd.ops import functional as Fx

    dy = torch.randn(256, 384, device="cuda").bfloat16()
    x = torch.randn(256, 128, device="cuda").bfloat16()
    assert not Fx._w4_dw_ok(256, 384, 128, dy, x)
    dw = Fx.weight_grad(dy, x, None)
    ref = dy.float().t() @ x.float()
    assert rel(dw, ref) < 1e-2


@pytest.mark.parametrize("ln", [False, True])
def test_add_norm_fused(ln):
    """AddNormFn on the GPU (fused residual add + norm, norm bwd with the residual grad fused)
    vs fp32 autograd of h = x + d, y = norm(h)."""
    from fault_tolerant_llm_training_amd.ops.functional import add_norm

    torch.manual_seed(3)
    M, N = 300, 4096
    x = torch.randn(M, N, device="cuda").bfloat16().requires_grad_(True)
    d = torch.randn(M, N, device="cuda").bfloat16().requires_grad_(True)
    w = (1 + 0.1 * torch.randn(N, device="cuda")).bfloat16().requires_grad_(True)
    h, y = add_norm(x, d, w, None, 1e-5, ln)
    dh = torch.randn(M, N, device="cuda").bfloat16()
    dy = torch.randn(M, N, device="cuda").bfloat16()
    torch.autograd.backward((h, y), (dh, dy))
    xr, dr, wr = (t.detach().float().requires_grad_(True) for t in (x, d, w))
    hr = xr + dr
    hc = hr - hr.mean(-1, keepdim=True) if ln else hr
    yr = hc * torch.rsqrt(hc.pow(2).mean(-1, keepdim=True) + 1e-5) * wr
    torch.autograd.backward((hr, yr), (dh.float(), dy.float()))
    assert rel(h, hr) < 1e-2 and rel(y, yr) < 1e-2
    assert rel(x.grad, xr.grad) < 2e-2 and torch.equal(x.grad, d.grad)
    assert rel(w.grad, wr.grad) < 2e-2


def test_pinned_ring_h2d():
    from fault_tolerant_llm_training_amd.ckpt.restore import h2d, release

    src = torch.randn(300 * (1 << 20) // 2).bfloat16()  # 300 MiB: > 1 chunk, ragged tail
    dst = torch.empty(src.numel(), dtype=torch.bfloat16, device="cuda")
    h2d(dst, src, min_bytes=0)
    torch.cuda.synchronize()
    assert torch.equal(dst.cpu(), src)
    release()


@pytest.mark.parametrize("w4", [False, True])
def test_feed_forward_fused(w4, monkeypatch):
    """The FFN node (GEMM -> SwiGLU -> GEMM, or every product on the w4 kernel with the SwiGLU
    epilogues: FeedForwardW4Fn), weight grads into sinks, vs fp32 autograd of
    w2(silu(x w1^T) * (x w3^T)) (reference model.py:254)."""
    from fault_tolerant_llm_training_amd.ops import functional as Fx
    from fault_tolerant_llm_training_amd.ops.grad_sink import GradSink

    if w4:
        monkeypatch.setattr(Fx, "_W4_MIN_TILES", 1)
        monkeypatch.setattr(Fx, "_W4_DEEP_K", 0)
    torch.manual_seed(5)
    T, D, Fh = 256, 256, 896  # F % 112 (SwiGLU tile), 2F % 256 (dW13 rows)
    x = torch.randn(T, D, device="cuda").bfloat16().requires_grad_(True)
    w13 = (0.05 * torch.randn(2 * Fh, D, device="cuda")).bfloat16()
    w2 = (0.05 * torch.randn(D, Fh, device="cuda")).bfloat16()
    assert Fx._ffn_w4t_ok(x.detach(), w13, w2) == w4
    g13 = torch.empty(w13.numel(), dtype=torch.bfloat16, device="cuda")
    g2 = torch.empty(w2.numel(), dtype=torch.bfloat16, device="cuda")
    y = Fx.feed_forward(x, w13, w2, GradSink(g13), GradSink(g2))
    dy = torch.randn(T, D, device="cuda").bfloat16()
    y.backward(dy)
    xr, w13r, w2r = (t.detach().float().requires_grad_(True) for t in (x, w13, w2))
    g, u = (xr @ w13r.t()).chunk(2, -1)
    yr = (F.silu(g) * u) @ w2r.t()
    yr.backward(dy.float())
    assert rel(y, yr) < 2e-2
    assert rel(x.grad, xr.grad) < 2e-2
    assert rel(g13.view(2 * Fh, D), w13r.grad) < 2e-2
    assert rel(g2.view(D, Fh), w2r.grad) < 2e-2


def test_h2d_from_checkpoint_file(tmp_path):
    """Restore path for an mmap'd checkpoint tensor: file -> pinned ring (native pread) -> HBM."""
    from fault_tolerant_llm_training_amd.ckpt import restore

    src = torch.randn(150 * (1 << 20) // 2).bfloat16()  # 150 MiB, ragged last chunk
    p = tmp_path / "ck.pt"
    torch.save({"x": src}, str(p))
    t = torch.load(str(p), mmap=True, weights_only=True)["x"]
    before = restore.STATS["file_bytes"]
    dst = torch.empty(src.numel(), dtype=torch.bfloat16, device="cuda")
    restore.h2d(dst, t, min_bytes=0)
    torch.cuda.synchronize()
    assert restore.STATS["file_bytes"] - before == src.numel() * 2
    assert torch.equal(dst.cpu(), src)
    restore.release()


def test_exact_math_switch(K):
    """AdamW / SwiGLU with the hardware v_rcp_f32 / v_sqrt_f32 (default) vs IEEE division and square
    root (FT_EXACT_MATH / set_exact_math): the bf16 results agree except for rare 1-ulp rounding flips."""
    torch.manual_seed(11)
    n = 1 << 20
    p = torch.randn(n, device="cuda").bfloat16()
    g = (torch.randn(n, device="cuda") * 1e-2).bfloat16()
    m = (torch.randn(n, device="cuda") * 1e-3).bfloat16()
    v = (torch.rand(n, device="cuda") * 1e-5).bfloat16()
    stats = torch.tensor([1.0, 1.0, 0.0], device="cuda")
    gu = torch.randn(2048, 2 * 1024, device="cuda").bfloat16()
    outs = {}
    try:
        for exact in (False, True):
            K.set_exact_math(exact)
            pp, mm, vv = p.clone(), m.clone(), v.clone()
            K.adamw_(pp, g, mm, vv, stats, 1e-3, 0.9, 0.999, 1e-8, 0.01, 7)
            outs[exact] = (pp, mm, vv, K.swiglu_fwd(gu))
    finally:
        K.set_exact_math(False)
    for a, b in zip(outs[False], outs[True]):
        diff = (a.float() - b.float()).abs()
        ulp = b.float().abs() * 2.0 ** -7 + 1e-30
        assert (diff <= ulp).all()
        assert (diff > 0).float().mean().item() < 0.02


@pytest.mark.parametrize("V,T,ntok,nparts", [(131072, 2048, 131072, 16384), (1000, 300, 40, 7), (5000, 4096, 3000, 300)])
def test_embedding_bwd_norm_partials(K, V, T, ntok, nparts):
    """embedding_bwd_ with partials (fresh gradient): the same gradient as without, every partial
    slot written (stale values cleared), their sum = the sum of squares of the stored gradient,
    bit-reproducible."""
    D = 256
    torch.manual_seed(V + T)
    tok = torch.randint(0, ntok, (T,), device="cuda")
    dy = torch.randn(T, D, device="cuda").bfloat16()
    ref = torch.zeros(V, D, device="cuda").bfloat16()
    K.embedding_bwd_(dy, tok, ref, False)
    dw = torch.full((V, D), 3.0, device="cuda").bfloat16()
    part = torch.full((nparts,), -5.0, device="cuda")
    K.embedding_bwd_(dy, tok, dw, False, part)
    assert torch.equal(dw, ref)
    want = ref.double().pow(2).sum().item()
    assert abs(part.double().sum().item() - want) <= 1e-5 * want
    assert torch.all(part >= 0)
    part2 = torch.zeros(nparts, device="cuda")
    K.embedding_bwd_(dy, tok, dw, False, part2)
    assert torch.equal(part2, part)
