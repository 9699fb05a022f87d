"""Llama-style decoder (the reference's only model family) with presets.

Math parity with reference ``model.py``: pre-norm residual blocks (:310-311),
RMSNorm with fp32 normalisation (:24-48), interleaved-pair RoPE (:100-126),
GQA causal attention (:179-215), SwiGLU FFN with the reference's hidden-size
rule (:243-247), untied LM head (:352). ``state_dict`` keys and parameter order
are identical to the reference (:170-177, :249-251, :291-292, :340, :350,
:352), so checkpoints load in both directions; the RoPE tables are
non-persistent buffers like ``freqs_cis`` (:342-344).

The execution path is MI355X-first: parameters are views into one flat HBM
buffer (``models.flat``), Q/K/V and W1/W3 run as single fused GEMMs against
adjacent-weight views, residual adds ride in the GEMM's C input, and every
non-GEMM op is a hand-written gfx950 kernel (``ops.functional``).
"""
from __future__ import annotations

from dataclasses import dataclass, replace
from typing import Optional

import torch
import torch.utils.checkpoint
import torch.nn as nn

from ..ops import functional as Fx
from .flat import FlatParamSpace


@dataclass
class TransformerModelArgs:
    """Same fields and defaults as reference ``TransformerModelArgs`` (model.py:9-21)."""

    dim: int = 4096
    n_layers: int = 32
    n_heads: int = 32
    n_kv_heads: Optional[int] = None
    multiple_of: int = 256
    ffn_dim_multiplier: Optional[float] = None
    norm_eps: float = 1e-5
    rope_theta: float = 10000
    norm_type: str = "rmsnorm"
    seq_len: int = 2048
    vocab_size: int = -1

    @property
    def kv_heads(self) -> int:
        return self.n_heads if self.n_kv_heads is None else self.n_kv_heads

    @property
    def head_dim(self) -> int:
        return self.dim // self.n_heads

    @property
    def ffn_hidden(self) -> int:
        """Reference FeedForward sizing (model.py:243-247) with hidden_dim = 4*dim."""
        hidden = int(2 * (4 * self.dim) / 3)
        if self.ffn_dim_multiplier is not None:
            hidden = int(self.ffn_dim_multiplier * hidden)
        return self.multiple_of * ((hidden + self.multiple_of - 1) // self.multiple_of)


# Presets. llama3-8b is the reference's hard-coded config (train.py:43-53).
# gpt2-small/medium are the BASELINE configs' sizes in the same Llama-style architecture.
PRESETS = {
    "llama3-8b": dict(dim=4096, n_layers=32, n_heads=32, n_kv_heads=8, ffn_dim_multiplier=1.3,
                      multiple_of=1024, rope_theta=500000),
    "gpt2-small": dict(dim=768, n_layers=12, n_heads=12, n_kv_heads=12, multiple_of=256,
                       rope_theta=10000),
    "gpt2-medium": dict(dim=1024, n_layers=24, n_heads=16, n_kv_heads=16, multiple_of=256,
                        rope_theta=10000),
    "tiny": dict(dim=256, n_layers=2, n_heads=4, n_kv_heads=2, multiple_of=64, rope_theta=10000),
}


def model_args_for(preset: str, vocab_size: int, seq_len: int, **overrides) -> TransformerModelArgs:
    if preset not in PRESETS:
        raise ValueError(f"unknown model preset {preset!r}; choose from {sorted(PRESETS)}")
    cfg = dict(PRESETS[preset])
    cfg.update(overrides)
    return TransformerModelArgs(vocab_size=vocab_size, seq_len=seq_len, **cfg)


def rope_tables(head_dim: int, end: int, theta: float):
    """cos/sin planes of the reference ``precompute_freqs_cis`` (model.py:51-71)."""
    freqs = 1.0 / (theta ** (torch.arange(0, head_dim, 2)[: (head_dim // 2)].float() / head_dim))
    t = torch.arange(end, device=freqs.device)
    freqs = torch.outer(t, freqs).float()
    cis = torch.polar(torch.ones_like(freqs), freqs)
    return cis.real.contiguous(), cis.imag.contiguous()


class _Weight(nn.Module):
    """Parameter holder with the reference's attribute name (``.weight``)."""

    def __init__(self, *shape):
        super().__init__()
        self.weight = nn.Parameter(torch.empty(*shape, device="meta"))


class Attention(nn.Module):
    def __init__(self, a: TransformerModelArgs):
        super().__init__()
        self.n_heads, self.n_kv_heads, self.head_dim = a.n_heads, a.kv_heads, a.head_dim
        self.wq = _Weight(a.n_heads * a.head_dim, a.dim)
        self.wk = _Weight(a.kv_heads * a.head_dim, a.dim)
        self.wv = _Weight(a.kv_heads * a.head_dim, a.dim)
        self.wo = _Weight(a.dim, a.n_heads * a.head_dim)
        self.wqkv = None  # fused view, set by bind_flat()
        self.wqkv_sink = None


class FeedForward(nn.Module):
    def __init__(self, a: TransformerModelArgs):
        super().__init__()
        h = a.ffn_hidden
        self.w1 = _Weight(h, a.dim)
        self.w2 = _Weight(a.dim, h)
        self.w3 = _Weight(h, a.dim)
        self.w13 = None
        self.w13_sink = None


class TransformerBlock(nn.Module):
    def __init__(self, layer_id: int, a: TransformerModelArgs):
        super().__init__()
        self.layer_id = layer_id
        self.attention = Attention(a)
        self.feed_forward = FeedForward(a)
        self.attention_norm = _Weight(a.dim)
        self.ffn_norm = _Weight(a.dim)
        self.eps = a.norm_eps
        self.layernorm = a.norm_type == "layernorm"
        self.attn_keep = Fx.AttentionKeep()

    def forward(self, h, d, cos, sin, seq_len, gen=None):
        """Pre-norm block (reference model.py:310-311) on the residual stream ``h`` with the
        previous block's pending output ``d`` (its add is fused into this block's first norm).
        Returns (h', d') with the block output h' + d' still to be added. ``gen``: the model's
        forward generation when this block is recomputed in backward with its attention output
        kept (selective checkpointing); None otherwise."""
        at, ff = self.attention, self.feed_forward
        sk = lambda p: getattr(p, "_ft_sink", None)  # noqa: E731
        if d is None:
            xn = Fx.norm(h, self.attention_norm.weight, sk(self.attention_norm.weight), self.eps, self.layernorm)
        else:
            h, xn = Fx.add_norm(h, d, self.attention_norm.weight, sk(self.attention_norm.weight), self.eps,
                                self.layernorm)
        o = Fx.qkv_rope_attention(xn, at.wqkv, at.wqkv_sink, cos, sin, seq_len, at.n_heads, at.n_kv_heads,
                                  at.head_dim, self.attn_keep if gen is not None else None, -1 if gen is None else gen)
        da = Fx.linear(o.view(*h.shape[:-1], -1), at.wo.weight, sk(at.wo.weight))
        h, hn = Fx.add_norm(h, da, self.ffn_norm.weight, sk(self.ffn_norm.weight), self.eps, self.layernorm)
        return h, Fx.feed_forward(hn, ff.w13, ff.w2.weight, ff.w13_sink, sk(ff.w2.weight))


class Transformer(nn.Module):
    def __init__(self, model_args: TransformerModelArgs):
        super().__init__()
        a = model_args
        self.model_args = a
        self.vocab_size = a.vocab_size
        self.n_layers = a.n_layers
        self.tok_embeddings = _Weight(a.vocab_size, a.dim)
        cos, sin = rope_tables(a.head_dim, a.seq_len, a.rope_theta)
        self.register_buffer("rope_cos", cos, persistent=False)
        self.register_buffer("rope_sin", sin, persistent=False)
        self.layers = nn.ModuleDict({str(i): TransformerBlock(i, a) for i in range(a.n_layers)})
        self.norm = _Weight(a.dim)
        self.output = _Weight(a.vocab_size, a.dim)
        self.flat: Optional[FlatParamSpace] = None
        self.gate = None  # optim.adamw.ParamGate: per-layer wait for the optimizer's updates
        self._ranges = None
        self.recompute_layers = 0  # activation checkpointing: blocks [0, n) recompute in backward
        self.recompute_attention = False  # False: recomputed blocks keep their attention output
        self._gen = 0  # forward generation (tags kept attention outputs)

    def set_activation_checkpointing(self, n_layers: int, recompute_attention: bool = False) -> None:
        """Recompute the first ``n_layers`` blocks (-1: all) during backward instead of keeping
        their activations: each block's input residual stream and — unless
        ``recompute_attention`` — its attention output and log-sum-exp stay resident, so the
        recompute runs the norms, projections, RoPE and FFN but not the flash forward (the
        O(S^2) part; T x Hq x D bf16 per block, 0.5 GB at seq 65536 for Llama-3-8B).
        Extends the reachable sequence length / batch per GPU (SURVEY.md §5.7 — the reference
        relies on SDPA's O(S) attention memory alone, model.py:212)."""
        self.recompute_layers = self.n_layers if n_layers < 0 else min(int(n_layers), self.n_layers)
        self.recompute_attention = bool(recompute_attention)

    # ------------------------------------------------------------------ materialisation
    def flat_layout(self):
        """Flat-buffer order: embedding, per layer [attention_norm | wq wk wv | wo | ffn_norm |
        w1 w3 | w2], head. Within a layer this is forward order, so backward produces the
        gradients at strictly descending addresses and the reducer's buckets (cut from the
        top down, launched in order) complete one after another."""
        names = ["tok_embeddings.weight"]
        for i in range(self.n_layers):
            p = f"layers.{i}."
            names += [p + "attention_norm.weight", p + "attention.wq.weight", p + "attention.wk.weight",
                      p + "attention.wv.weight", p + "attention.wo.weight", p + "ffn_norm.weight",
                      p + "feed_forward.w1.weight", p + "feed_forward.w3.weight", p + "feed_forward.w2.weight"]
        names += ["norm.weight", "output.weight"]
        return names

    def materialize(self, device, dtype=torch.bfloat16, seed: int = 1234) -> "Transformer":
        """Allocate the flat buffers on ``device`` and initialise like the reference.

        Initialisation happens directly on the device (the reference builds the
        8B model on the CPU, ~35 s of its setup — SURVEY.md §A.8).
        """
        self.flat = FlatParamSpace(self, self.flat_layout(), device, dtype)
        self.rope_cos = self.rope_cos.to(device)
        self.rope_sin = self.rope_sin.to(device)
        for layer in self.layers.values():
            at, ff = layer.attention, layer.feed_forward
            i = layer.layer_id
            at.wqkv, at.wqkv_sink = self.flat.fused(
                [f"layers.{i}.attention.wq.weight", f"layers.{i}.attention.wk.weight", f"layers.{i}.attention.wv.weight"])
            ff.w13, ff.w13_sink = self.flat.fused(
                [f"layers.{i}.feed_forward.w1.weight", f"layers.{i}.feed_forward.w3.weight"])
        self._ranges = self._param_ranges()
        self.init_weights(seed)
        return self

    def _param_ranges(self):
        """Flat [lo, hi) of the weights used by: embedding, each layer, final norm + head."""
        sl = self.flat.slots

        def span(prefix):
            ss = [s for n, s in sl.items() if n.startswith(prefix)]
            return min(s.offset for s in ss), max(s.offset + s.numel for s in ss)

        emb = span("tok_embeddings.")
        layers = [span(f"layers.{i}.") for i in range(self.n_layers)]
        lo_n, hi_n = span("norm.")
        lo_o, hi_o = span("output.")
        return emb, layers, (min(lo_n, lo_o), max(hi_n, hi_o))

    def _wait(self, rng):
        if self.gate is not None:
            self.gate.wait(*rng)

    @torch.no_grad()
    def init_weights(self, seed: int = 1234):
        """nn.Linear default (U(±1/sqrt(fan_in))), nn.Embedding N(0,1), norms = 1 (reference init)."""
        dev = self.flat.device
        gen = torch.Generator(device=dev)
        for idx, (name, p) in enumerate(self.named_parameters()):
            gen.manual_seed(seed * 1000003 + idx)
            if name == "tok_embeddings.weight":
                p.normal_(0.0, 1.0, generator=gen)
            elif p.dim() == 1:
                p.fill_(1.0)
            else:
                bound = 1.0 / (p.shape[1] ** 0.5)
                p.uniform_(-bound, bound, generator=gen)

    def sinks_in_backward_order(self):
        """Fused-view sinks used by the forward (for DDP readiness accounting)."""
        out = []
        for layer in self.layers.values():
            out += [layer.attention.wqkv_sink, layer.feed_forward.w13_sink]
        return out

    # ------------------------------------------------------------------ forward
    def forward(self, tokens: torch.Tensor, labels: Optional[torch.Tensor] = None,
                inv_count: Optional[torch.Tensor] = None):
        """tokens: [B, S] int64. With labels: returns the scalar loss
        (sum of token NLL × inv_count, reference train.py:101-102); else logits."""
        B, S = tokens.shape
        sk = lambda p: getattr(p, "_ft_sink", None)  # noqa: E731
        emb_r, layer_r, final_r = self._ranges
        self._wait(emb_r)
        h = Fx.embedding(tokens, self.tok_embeddings.weight, sk(self.tok_embeddings.weight))
        cos, sin = self.rope_cos, self.rope_sin
        d = None
        self._gen += 1
        gen = None if self.recompute_attention else self._gen
        for i, layer in enumerate(self.layers.values()):
            self._wait(layer_r[i])
            if i < self.recompute_layers and torch.is_grad_enabled():
                # non-reentrant: the custom Functions' saved tensors are dropped and regenerated
                # by re-running the block (deterministic kernels → bit-identical gradients);
                # with ``gen`` the re-run reuses the kept attention output
                h, d = torch.utils.checkpoint.checkpoint(layer, h, d, cos, sin, S, gen, use_reentrant=False)
            else:
                h, d = layer(h, d, cos, sin, S)
        self._wait(final_r)
        a = self.model_args
        ln = a.norm_type == "layernorm"
        if d is None:
            h = Fx.norm(h, self.norm.weight, sk(self.norm.weight), a.norm_eps, ln)
        else:
            _, h = Fx.add_norm(h, d, self.norm.weight, sk(self.norm.weight), a.norm_eps, ln)
        if labels is None:
            return Fx.linear(h, self.output.weight, sk(self.output.weight))
        if inv_count is None:
            n = (labels != Fx.IGNORE_INDEX).sum().clamp(min=1)
            inv_count = (1.0 / n.float()).to(h.device)
        return Fx.lm_head_cross_entropy(h, self.output.weight, labels, inv_count, sk(self.output.weight))

    def num_params(self) -> int:
        return sum(p.numel() for p in self.parameters())


def build_model(args: TransformerModelArgs, device, dtype=torch.bfloat16, seed: int = 1234) -> Transformer:
    return Transformer(args).materialize(device, dtype, seed)


# Dense matrix-core peaks of one MI355X per model dtype (no 2:1 sparsity): the MFU denominator
PEAK_FLOPS = {torch.bfloat16: 2.5e15, torch.float16: 2.5e15, torch.float32: 157.3e12, torch.float64: 78.6e12}


def flops_per_token(a: TransformerModelArgs, seq_len: int) -> float:
    """Training FLOPs/token: 6 × matmul params + causal attention (fwd+bwd = 3 × fwd)."""
    d, L, hd = a.dim, a.n_layers, a.head_dim
    per_layer = d * (a.n_heads * hd) + 2 * d * (a.kv_heads * hd) + (a.n_heads * hd) * d + 3 * d * a.ffn_hidden
    n_mm = L * per_layer + d * a.vocab_size
    attn = L * 2 * 2 * seq_len * a.n_heads * hd / 2  # QK^T + PV, causal half, per token
    return 6 * n_mm + 3 * attn
