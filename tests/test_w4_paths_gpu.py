"""The model's w4-kernel backward paths end to end, on a small model driven through them.

The w4 routing only takes products with at least half the chip in output tiles (and the fused
QKV + RoPE projection only from model dim 2048), so the tiny / GPT-2 GPU tests never reach it.
Here those gates are lowered (``_W4_MIN_TILES``, ``_W4_DEEP_K``, ``_QKV_ROPE_MIN_K``) and a Llama-style model
whose FFN width is a multiple of 112 (the SwiGLU-epilogue tile) runs:
  forward  QKV GEMM with the RoPE epilogue, wo / w2 with the residual epilogue, w1|w3 with the
           SwiGLU epilogue, the LM head on the w4 kernel
  backward QKVRopeFn (RoPE rotated back in place, then dW / dX on k-major operands),
           FeedForwardW4Fn (dW2, da with the SwiGLU-backward epilogue, dW13, dX), the head's
           dX / dW, every dW with its gradient-norm partials in the epilogue.
Loss and every gradient are compared with the fp32 CPU model on the same weights, and with the
same GPU model on the round-3 routing (hipBLASLt backward); the fused sums of squares must add up
to the gradient's norm with the separate pass run only for the embedding.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu


def rel(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm()).item()


@pytest.fixture
def gates(monkeypatch):
    from fault_tolerant_llm_training_amd.ops import functional as Fx

    monkeypatch.setattr(Fx, "_W4_MIN_TILES", 1)

    monkeypatch.setattr(Fx, "_W4_DEEP_K", 0)
    from fault_tolerant_llm_training_amd.ops import attention as A

    monkeypatch.setattr(A, "_QKV_ROPE_MIN_K", 0)
    return Fx


def _args(V=4096, S=512):
    from fault_tolerant_llm_training_amd.models.llama import TransformerModelArgs

    # dim 512, 8 heads of 64, 4 KV heads, FFN 1792 (= 16 x 112; multiple_of rounds 1365 up to it)
    return TransformerModelArgs(dim=512, n_layers=2, n_heads=8, n_kv_heads=4, multiple_of=1792,
                                rope_theta=10000, vocab_size=V, seq_len=S)


def _step(m, tok, lab):
    loss = m(tok, lab)
    loss.backward()
    return loss.detach()


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
def test_w4_paths_vs_cpu_and_blas(gates, dt):
    from fault_tolerant_llm_training_amd.models.llama import build_model
    from fault_tolerant_llm_training_amd.ops import attention as A

    Fx = gates
    a = _args()
    assert a.ffn_hidden == 1792
    mg = build_model(a, "cuda", dt, seed=11)
    mc = build_model(a, "cpu", torch.float32, seed=11)
    mc.load_state_dict({k: v.float().cpu() for k, v in mg.state_dict().items()})
    torch.manual_seed(5)
    tok = torch.randint(0, a.vocab_size, (1, a.seq_len))
    lab = torch.randint(0, a.vocab_size, (1, a.seq_len))
    x2 = torch.empty(a.seq_len, a.dim, device="cuda", dtype=dt)
    w13 = mg.layers["0"].feed_forward.w13
    w2 = mg.layers["0"].feed_forward.w2.weight
    assert Fx._ffn_w4t_ok(x2, w13, w2)  # the FFN really takes FeedForwardW4Fn
    assert A._qkv_rope_ok(x2, mg.layers["0"].attention.wqkv, a.head_dim)
    lg = _step(mg, tok.cuda(), lab.cuda())
    g_w4 = mg.flat.grads.clone()
    lc = _step(mc, tok, lab)
    assert abs(lg.item() - lc.item()) < 5e-3 * abs(lc.item())
    assert rel(g_w4.cpu(), mc.flat.grads) < 3e-2
    # the same GPU model on the round-3 routing: hipBLASLt backward, separate RoPE / SwiGLU passes
    Fx.set_w4_bwd(False)
    Fx.set_qkv_rope(False)
    Fx.set_w4_swiglu(False)
    try:
        mg.flat.grads.zero_()
        lb = _step(mg, tok.cuda(), lab.cuda())
    finally:
        Fx.set_w4_bwd(True)
        Fx.set_qkv_rope(True)
        Fx.set_w4_swiglu(True)
    assert abs(lb.item() - lg.item()) < 2e-3 * abs(lb.item())
    assert rel(g_w4, mg.flat.grads) < 2e-2
    # per parameter too: no gradient may be wrong while the total looks fine
    for name, s in mg.flat.slots.items():
        g1 = g_w4[s.offset: s.offset + s.numel]
        gc = mc.flat.grads[s.offset: s.offset + s.numel]
        if gc.norm() > 0:
            assert rel(g1.cpu(), gc) < 5e-2, name


def test_fused_sumsq_partials(gates, monkeypatch):
    """Local-mode reducer: the w4 dW / head epilogues, the norm backward and the embedding backward
    (rows it stores; every other row is zero) write the norm partials: no separate sumsq pass runs,
    and the total equals the gradient's sum of squares."""
    from fault_tolerant_llm_training_amd.models.llama import build_model
    from fault_tolerant_llm_training_amd.parallel import ddp

    calls = []
    real = ddp.kernels()

    class Spy:
        def __getattr__(self, n):
            f = getattr(real, n)
            if n == "sumsq_into_":
                def g(grad, part):
                    calls.append(grad.numel())
                    return f(grad, part)
                return g
            return f

    monkeypatch.setattr(ddp, "kernels", lambda: Spy())
    a = _args()
    m = build_model(a, "cuda", torch.bfloat16, seed=3)
    red = ddp.GradReducer(m.flat, m.sinks_in_backward_order(), bucket_mb=1.0)
    assert red.fused_sumsq
    torch.manual_seed(1)
    tok = torch.randint(0, a.vocab_size, (1, a.seq_len), device="cuda")
    for it in range(2):  # the flags reset between steps
        calls.clear()
        red.begin_micro(0, 1)
        m(tok, tok).backward()
        red.finish()
        torch.cuda.synchronize()
        want = m.flat.grads.double().pow(2).sum().item()
        got = red.global_sumsq().double().sum().item()
        assert abs(got - want) <= 2e-5 * want, (it, got, want)
        assert calls == [], calls


def test_fused_sumsq_fallback_runs_merged(monkeypatch):
    """Without producer partials (the hipBLASLt backward, as for the small presets) every sink
    falls back to the sum-of-squares pass: adjacent sinks of a bucket take one launch, the total
    still equals the gradient's sum of squares."""
    from fault_tolerant_llm_training_amd.models.llama import build_model
    from fault_tolerant_llm_training_amd.ops import functional as Fx
    from fault_tolerant_llm_training_amd.parallel import ddp

    monkeypatch.setattr(Fx, "_W4_BWD", False)
    calls = []
    real = ddp.kernels()

    class Spy:
        def __getattr__(self, n):
            f = getattr(real, n)
            if n == "sumsq_into_":
                def g(grad, part):
                    calls.append(grad.numel())
                    return f(grad, part)
                return g
            return f

    monkeypatch.setattr(ddp, "kernels", lambda: Spy())
    a = _args()
    m = build_model(a, "cuda", torch.bfloat16, seed=3)
    red = ddp.GradReducer(m.flat, m.sinks_in_backward_order(), bucket_mb=1.0)
    assert red.fused_sumsq
    torch.manual_seed(1)
    tok = torch.randint(0, a.vocab_size, (1, a.seq_len), device="cuda")
    for it in range(2):
        calls.clear()
        red.begin_micro(0, 1)
        m(tok, tok).backward()
        red.finish()
        torch.cuda.synchronize()
        want = m.flat.grads.double().pow(2).sum().item()
        got = red.global_sumsq().double().sum().item()
        assert abs(got - want) <= 2e-5 * want, (it, got, want)
        fallback = [s for s in red._sq_sinks if s.part is not None]
        assert 0 < len(calls) < len(fallback), (len(calls), len(fallback))
        assert sum(calls) <= m.flat.grads.numel()


def test_fused_sumsq_fallback_then_producer(gates):
    """A step whose sinks took the fallback pass (producer partials off: every slot of a sink's slice
    written) followed by steps with the w4 dW epilogue partials (fewer tiles than slots): the slots
    past the tile grid must not keep the fallback's values, or the global norm is inflated."""
    from fault_tolerant_llm_training_amd.models.llama import build_model
    from fault_tolerant_llm_training_amd.parallel import ddp

    a = _args()
    m = build_model(a, "cuda", torch.bfloat16, seed=3)
    red = ddp.GradReducer(m.flat, m.sinks_in_backward_order(), bucket_mb=1.0)
    assert red.fused_sumsq
    torch.manual_seed(2)
    for it, producers in enumerate([False, True, True]):
        torch.cuda.synchronize()
        red.set_producer_sums(producers)
        tok = torch.randint(0, a.vocab_size, (1, a.seq_len), device="cuda")
        red.begin_micro(0, 1)
        # a loss scale that changes per step, so a stale partial cannot match by accident (powers
        # of two: the fused head's partials are of its unscaled dW times g^2, exact only then)
        (m(tok, tok) * float(4 ** it)).backward()
        red.finish()
        torch.cuda.synchronize()
        want = m.flat.grads.double().pow(2).sum().item()
        got = red.global_sumsq().double().sum().item()
        assert abs(got - want) <= 2e-5 * want, (it, producers, got, want)
