"""Model math vs an independent eager implementation of the reference's model.py.

The reference model (model.py:24-380): RMSNorm in fp32 then ``type_as`` then ×weight,
complex-multiply RoPE on interleaved pairs, materialised repeat_kv, causal SDPA,
SwiGLU ``w2(silu(w1 x) * w3 x)``, untied head; loss = CE(sum)/num_items
(train.py:101-102). Parameters are loaded through the shared state_dict keys.
"""
import math

import pytest
import torch
import torch.nn.functional as F

from fault_tolerant_llm_training_amd.models.llama import build_model, model_args_for


def ref_forward(sd, a, tokens):
    def rms(x, w):
        xf = x.float()
        return (xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + a.norm_eps)).type_as(x) * w

    hd = a.dim // a.n_heads
    kv = a.kv_heads
    freqs = 1.0 / (a.rope_theta ** (torch.arange(0, hd, 2)[: hd // 2].float() / hd))
    cis = torch.polar(torch.ones(a.seq_len, hd // 2), torch.outer(torch.arange(a.seq_len).float(), freqs))

    def rope(x):
        B, S, H, D = x.shape
        xc = torch.view_as_complex(x.float().reshape(B, S, H, D // 2, 2))
        return torch.view_as_real(xc * cis[:S].view(1, S, 1, D // 2)).flatten(3).type_as(x)

    h = sd["tok_embeddings.weight"][tokens]
    B, S = tokens.shape
    for i in range(a.n_layers):
        p = f"layers.{i}."
        x = rms(h, sd[p + "attention_norm.weight"])
        q = (x @ sd[p + "attention.wq.weight"].t()).view(B, S, a.n_heads, hd)
        k = (x @ sd[p + "attention.wk.weight"].t()).view(B, S, kv, hd)
        v = (x @ sd[p + "attention.wv.weight"].t()).view(B, S, kv, hd)
        q, k = rope(q), rope(k)
        rep = a.n_heads // kv
        k = k[:, :, :, None, :].expand(B, S, kv, rep, hd).reshape(B, S, a.n_heads, hd)
        v = v[:, :, :, None, :].expand(B, S, kv, rep, hd).reshape(B, S, a.n_heads, hd)
        o = F.scaled_dot_product_attention(q.transpose(1, 2), k.transpose(1, 2), v.transpose(1, 2), is_causal=True)
        o = o.transpose(1, 2).reshape(B, S, -1)
        h = h + o @ sd[p + "attention.wo.weight"].t()
        x = rms(h, sd[p + "ffn_norm.weight"])
        g = F.silu(x @ sd[p + "feed_forward.w1.weight"].t()) * (x @ sd[p + "feed_forward.w3.weight"].t())
        h = h + g @ sd[p + "feed_forward.w2.weight"].t()
    h = rms(h, sd["norm.weight"])
    return h @ sd["output.weight"].t()


def test_state_dict_keys_match_reference_layout():
    a = model_args_for("tiny", vocab_size=128, seq_len=16)
    m = build_model(a, "cpu", torch.float32, seed=0)
    keys = list(m.state_dict().keys())
    exp = ["tok_embeddings.weight"]
    for i in range(a.n_layers):
        p = f"layers.{i}."
        exp += [p + "attention.wq.weight", p + "attention.wk.weight", p + "attention.wv.weight",
                p + "attention.wo.weight", p + "feed_forward.w1.weight", p + "feed_forward.w2.weight",
                p + "feed_forward.w3.weight", p + "attention_norm.weight", p + "ffn_norm.weight"]
    exp += ["norm.weight", "output.weight"]
    assert keys == exp
    assert not any("rope" in k or "freqs" in k for k in keys)  # non-persistent tables


def test_llama3_8b_shapes():
    a = model_args_for("llama3-8b", vocab_size=131072, seq_len=2048)
    assert a.ffn_hidden == 14336  # reference model.py:243-247 rule
    assert a.head_dim == 128 and a.kv_heads == 8
    per_layer = 4096 * 4096 * 2 + 2 * 4096 * 1024 + 3 * 4096 * 14336 + 2 * 4096
    total = 32 * per_layer + 2 * 131072 * 4096 + 4096
    assert abs(total / 1e9 - 8.053) < 0.001  # 8.05 B


@pytest.mark.parametrize("preset", ["tiny"])
def test_forward_backward_matches_reference_math(preset):
    torch.manual_seed(0)
    a = model_args_for(preset, vocab_size=257, seq_len=24)
    m = build_model(a, "cpu", torch.float32, seed=3)
    tok = torch.randint(0, 257, (2, 24))
    lab = torch.randint(0, 257, (2, 24))
    lab[0, :3] = -100
    sd = {k: v.detach().clone().requires_grad_(True) for k, v in m.state_dict().items()}
    logits_ref = ref_forward(sd, a, tok)
    n = (lab != -100).sum()
    loss_ref = F.cross_entropy(logits_ref.flatten(0, 1).float(), lab.flatten(), reduction="sum") / n
    loss_ref.backward()
    logits = m(tok)
    assert torch.allclose(logits, logits_ref, atol=1e-4, rtol=1e-4)
    loss = m(tok, lab)
    assert math.isclose(loss.item(), loss_ref.item(), rel_tol=1e-5)
    loss.backward()
    named = dict(m.named_parameters())
    for k, v in sd.items():
        assert torch.allclose(named[k].grad, v.grad, atol=1e-5, rtol=1e-4), k


def test_layernorm_variant():
    a = model_args_for("tiny", vocab_size=64, seq_len=8, norm_type="layernorm")
    m = build_model(a, "cpu", torch.float32, seed=1)
    tok = torch.randint(0, 64, (1, 8))
    loss = m(tok, tok)
    loss.backward()
    assert torch.isfinite(loss)
    assert m.flat.grads.abs().sum() > 0


@pytest.mark.parametrize("recompute_attention", [False, True])
@pytest.mark.parametrize("n", [1, -1])
def test_activation_checkpointing_same_loss_and_grads(n, recompute_attention):
    """Recomputing blocks in backward (--activation-checkpointing), with or without keeping the
    attention output, changes nothing."""
    a = model_args_for("tiny", vocab_size=128, seq_len=32)
    tok = torch.randint(0, 128, (2, 32))
    lab = torch.randint(0, 128, (2, 32))
    out = []
    for k in (0, n):
        m = build_model(a, "cpu", torch.float32, seed=5)
        m.set_activation_checkpointing(k, recompute_attention=recompute_attention)
        loss = m(tok, lab)
        loss.backward()
        out.append((loss.detach(), m.flat.grads.clone()))
    assert m.recompute_layers == (a.n_layers if n < 0 else n)
    assert torch.equal(out[0][0], out[1][0])
    assert torch.allclose(out[0][1], out[1][1], rtol=0, atol=1e-6)


def test_selective_checkpointing_skips_attention_recompute(monkeypatch):
    """Kept attention outputs: the backward recompute runs no attention forward, a forward whose
    backward never ran leaves nothing stale, and gradients match the no-recompute model."""
    from fault_tolerant_llm_training_amd.ops import attention as A

    calls = []
    real = A.attention_reference
    monkeypatch.setattr(A, "attention_reference", lambda *x: calls.append(1) or real(*x))
    a = model_args_for("tiny", vocab_size=128, seq_len=32)
    tok = torch.randint(0, 128, (2, 32))
    lab = torch.randint(0, 128, (2, 32))
    ref = build_model(a, "cpu", torch.float32, seed=5)
    ref(tok, lab).backward()
    for recompute_attention, per_step in ((False, a.n_layers), (True, 2 * a.n_layers)):
        m = build_model(a, "cpu", torch.float32, seed=5)
        m.set_activation_checkpointing(-1, recompute_attention=recompute_attention)
        m(tok[:, :16], lab[:, :16])  # forward only (no backward): its kept outputs go stale
        calls.clear()
        m(tok, lab).backward()
        # the CPU backward of attention re-derives it under autograd: one call per block
        assert len(calls) == per_step + a.n_layers
        assert torch.allclose(m.flat.grads, ref.flat.grads, rtol=0, atol=1e-6)
        assert all(l.attn_keep.o is None for l in m.layers.values()) or recompute_attention


@pytest.mark.parametrize("solo", ["1", "0"])
def test_embedding_solo_bucket_on_one_rank(solo, monkeypatch):
    """On one rank the token-embedding table gets an optimizer bucket of its own (the next forward
    waits only for the table's AdamW); FT_EMB_SOLO_BUCKET=0 restores the plain size cut. Either
    way the buckets tile the flat buffer exactly."""
    from fault_tolerant_llm_training_amd.models.llama import build_model, model_args_for
    from fault_tolerant_llm_training_amd.parallel.ddp import GradReducer

    monkeypatch.setenv("FT_EMB_SOLO_BUCKET", solo)
    m = build_model(model_args_for("tiny", vocab_size=512, seq_len=32), "cpu", torch.bfloat16, seed=0)
    red = GradReducer(m.flat, m.sinks_in_backward_order(), bucket_mb=1.0)
    spans = sorted((b.lo, b.hi) for b in red.buckets)
    assert spans[0][0] == 0 and spans[-1][1] == m.flat.numel
    assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
    es = m.flat.slots["tok_embeddings.weight"]
    own = any(b.lo == es.offset and b.hi == es.offset + es.numel for b in red.buckets)
    assert own == (solo == "1")
