"""Causal GQA flash attention on packed projections (gfx950 HIP kernels).

Q and K come rotated (reference model.py:100-126) from one of two producers:
by default the QKV projection's GEMM epilogue (``gemm_qkv_rope_w4``, csrc/kernels/gemm_w4.hip)
rotates them in place, so ``qk`` IS the packed ``qkv`` projection ``[T, (Hq+2Hkv)*D]``; on the
paths without that epilogue (fp32, GPT-2-sized models, set_qkv_rope(False)) the RoPE kernel
(csrc/kernels/rope.hip) writes a separate rotated ``qk`` buffer ``[T, (Hq+Hkv)*D]``. V is always
read in place from ``qkv``. KV heads are indexed as ``h // (Hq/Hkv)`` inside the kernels, so
the reference's materialised ``repeat_kv`` (model.py:129-138) and the transpose/contiguous
copies (model.py:207-213) never exist. This module picks the kernel family by dtype
(bf16/fp16: csrc/kernels/flash_attn.hip, fp32: csrc/kernels/flash_f32.hip) and exposes the
deterministic / non-deterministic backward switch; and the autograd functions of RoPE +
attention on the packed projection (reference model.py:179-215).
"""
from __future__ import annotations

import os
from typing import Optional

import torch
import torch.nn.functional as F

from .._native import kernels, native

# Backward variant: 1 = deterministic (default): KV-major dK/dV kernel + Q-major dQ
# kernel, no atomics, bit-reproducible — GPU resume is bit-exact with it and it runs
# as fast as 0 = dQ accumulated with fp32 atomics in the KV-major kernel (Llama-3-8B
# layer shape: profiles/r1_flash_kernels.md).
_BWD_MODE = int(os.environ.get("FT_FLASH_BWD_MODE", "1"))


def set_deterministic(flag: bool) -> None:
    global _BWD_MODE
    _BWD_MODE = 1 if flag else 0


def flash_attn_fwd(qk, qkv, S, hq, hkv, d):
    """Returns (o [T, Hq*D], lse [B, Hq, S'] fp32) in the model dtype. The HIP kernels only, no
    fallback (``kernels()`` raises if the extension is missing): the MFMA kernels for bf16 / fp16
    (csrc/kernels/flash_attn.hip), the fp32 vector-ALU kernels for fp32 models (flash_f32.hip)."""
    if qk.dtype == torch.float32:
        return tuple(kernels().flash_f32_fwd(qk, qkv, S, hq, hkv, d))
    return tuple(kernels().flash_fwd(qk, qkv, S, hq, hkv, d))


def flash_attn_bwd(do, qk, qkv, o, lse, S, hq, hkv, d, cos=None, sin=None):
    """Returns dqkv [T, (Hq+2Hkv)*D]. With ``cos`` / ``sin`` the dQ / dK columns are rotated back
    (RoPE backward, reference model.py:100-126): the gradient of the UNROTATED projection — on the
    16-bit path inside the kernel pass that folds the GQA dK / dV partials (no separate RoPE
    pass); without them dQ / dK stay in the rotated frame. Both variants are deterministic (fp32:
    always; bf16 / fp16: unless FT_FLASH_BWD_MODE=0)."""
    if qk.dtype == torch.float32:
        dqkv = kernels().flash_f32_bwd(do, qk, qkv, o, lse, S, hq, hkv, d)
        if cos is not None:
            kernels().rope_bwd_(dqkv, cos, sin, S, hq, hkv, d)
        return dqkv
    return kernels().flash_bwd(do, qk, qkv, o, lse, S, hq, hkv, d, _BWD_MODE, cos, sin)


# --------------------------------------------------------------------------------------
# RoPE + causal GQA attention on the fused QKV projection (autograd)
# --------------------------------------------------------------------------------------


def rope_reference(x: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor) -> torch.Tensor:
    """x: [B, S, H, D] interleaved pairs; cos/sin: [S, D/2] fp32."""
    xf = x.float().reshape(*x.shape[:-1], -1, 2)
    a, b = xf[..., 0], xf[..., 1]
    c = cos[: x.shape[1]].view(1, x.shape[1], 1, -1)
    s = sin[: x.shape[1]].view(1, x.shape[1], 1, -1)
    out = torch.stack((a * c - b * s, a * s + b * c), dim=-1).flatten(-2)
    return out.type_as(x)


def attention_reference(qkv, cos, sin, seq_len, hq, hkv, d):
    """Reference math: RoPE → repeat_kv → causal SDPA (model.py:179-215). qkv: [B*S, W]."""
    T = qkv.shape[0]
    B = T // seq_len
    q = qkv[:, : hq * d].reshape(B, seq_len, hq, d)
    k = qkv[:, hq * d : (hq + hkv) * d].reshape(B, seq_len, hkv, d)
    v = qkv[:, (hq + hkv) * d :].reshape(B, seq_len, hkv, d)
    q = rope_reference(q, cos, sin)
    k = rope_reference(k, cos, sin)
    rep = hq // hkv
    if rep > 1:
        k = k.repeat_interleave(rep, dim=2)
        v = v.repeat_interleave(rep, dim=2)
    o = F.scaled_dot_product_attention(q.transpose(1, 2), k.transpose(1, 2), v.transpose(1, 2), is_causal=True)
    return o.transpose(1, 2).reshape(T, hq * d)


class AttentionKeep:
    """Per-block holder of the attention output kept across a recomputed block (selective
    activation checkpointing): the first forward of a checkpointed block stores (o, lse) here
    tagged with the model's forward generation; the recompute in backward (same generation)
    reuses them instead of running the flash forward again. A stale entry (a forward whose
    backward never ran) carries an older generation and is simply overwritten."""

    __slots__ = ("gen", "o", "lse")

    def __init__(self):
        self.gen, self.o, self.lse = -1, None, None


class RopeAttentionFn(torch.autograd.Function):
    """RoPE + causal GQA attention on the packed projection. ``rotated``: Q/K of ``qkv`` were
    already rotated by the QKV projection's epilogue (:class:`QKVRopeFn`, GPU only): the flash
    kernels then read Q/K straight from ``qkv``. Either way backward returns the gradient of the
    UNROTATED projection: the flash backward rotates dQ/dK back in the pass that folds the GQA
    dK/dV partials (so neither this node nor the projection's backward runs a RoPE pass)."""

    @staticmethod
    def forward(ctx, qkv, cos, sin, seq_len, hq, hkv, d, keep=None, gen=-1, rotated=False):
        ctx.cfg = (seq_len, hq, hkv, d)
        ctx.rotated = rotated
        hit = keep is not None and keep.gen == gen and keep.o is not None
        if native(qkv):
            qkv = qkv.contiguous()
            qk = qkv if rotated else kernels().rope_fwd(qkv, cos, sin, seq_len, hq, hkv, d)
            if hit:  # recompute pass of a checkpointed block: the kept output (bit-identical)
                o, lse = keep.o, keep.lse
                keep.o = keep.lse = None
            else:
                o, lse = flash_attn_fwd(qk, qkv, seq_len, hq, hkv, d)
                if keep is not None:
                    keep.gen, keep.o, keep.lse = gen, o, lse
            ctx.save_for_backward(qkv, qk, o, lse, cos, sin)
            return o
        ctx.save_for_backward(qkv, cos, sin)
        if hit:
            o = keep.o
            keep.o = None
        else:
            o = attention_reference(qkv, cos, sin, seq_len, hq, hkv, d)
            if keep is not None:
                keep.gen, keep.o = gen, o
        return o

    @staticmethod
    def backward(ctx, do):
        seq_len, hq, hkv, d = ctx.cfg
        if native(do):
            qkv, qk, o, lse, cos, sin = ctx.saved_tensors
            dqkv = flash_attn_bwd(do.contiguous(), qk, qkv, o, lse, seq_len, hq, hkv, d, cos, sin)
            return dqkv, None, None, None, None, None, None, None, None, None
        qkv, cos, sin = ctx.saved_tensors
        with torch.enable_grad():
            x = qkv.detach().requires_grad_(True)
            o = attention_reference(x, cos, sin, seq_len, hq, hkv, d)
            (dx,) = torch.autograd.grad(o, (x,), do)
        return dx, None, None, None, None, None, None, None, None, None


def rope_attention(qkv, cos, sin, seq_len, hq, hkv, d, keep: Optional[AttentionKeep] = None, gen: int = -1,
                   rotated: bool = False):
    """RoPE on the packed projection, then causal GQA attention. ``keep``/``gen``: selective
    activation checkpointing (see :class:`AttentionKeep`)."""
    return RopeAttentionFn.apply(qkv, cos, sin, seq_len, hq, hkv, d, keep, gen, rotated)


# QKV projection with RoPE in the GEMM epilogue (csrc/kernels/gemm_w4.hip, gemm_qkv_rope_w4): the
# hand-written 4-wave GEMM writes qkv with Q/K already rotated, so neither the separate RoPE
# kernel nor the rotated [T, (Hq + Hkv) D] copy exists; the flash kernels read Q/K from qkv.
# Default on (8B step: 1.001-1.003x, the RoPE forward kernel and the rotated copy gone; the
# kernel alone runs the Llama-3-8B QKV shape at 1.10-1.14x hipBLASLt, profiles/r3_gemm_w4_investigation.md);
# set_qkv_rope(False) restores the plain projection + the RoPE kernel (A/B).
_QKV_ROPE = True
# model dim from which the fused projection wins (see _qkv_rope_ok; FT_QKV_ROPE_MIN_K: A/B)
_QKV_ROPE_MIN_K = int(os.environ.get("FT_QKV_ROPE_MIN_K", "2048"))


def set_qkv_rope(on: bool) -> None:
    global _QKV_ROPE
    _QKV_ROPE = bool(on)


def _qkv_rope_ok(x2: torch.Tensor, w: torch.Tensor, d: int) -> bool:
    if not (_QKV_ROPE and Fx._W4_FWD and w.is_contiguous()):
        return False
    # K >= 2048 (the 8B-class projections): at GPT-2 sizes (K = 768 / 1024) the epilogue kernel
    # loses ~1 % of the step to hipBLASLt + the RoPE kernel (profiles/r3_gpt2_w4_ab.log). The
    # kernel takes no K split: the tile grid alone must fill half the chip.
    T, K = x2.shape
    N = w.shape[0]
    if d % 8 or K < _QKV_ROPE_MIN_K or not Fx.w4_route(T, N, K, False, False, x2, w):
        return False
    nj = kernels().gemm_w4_pick(T, N)
    return nj > 0 and (T // 256) * (N // (32 * nj)) >= Fx._W4_MIN_TILES


class QKVRopeFn(torch.autograd.Function):
    """qkv = x W^T with Q/K rotated (reference model.py:195 then :100-126). Backward receives the
    gradient of the unrotated projection (the attention backward already rotated dQ/dK back,
    :class:`RopeAttentionFn`), then dW / dX."""

    @staticmethod
    def forward(ctx, x2, w, sink, cos, sin, seq_len, hq, hkv, d):
        ctx.sink = sink
        ctx.cfg = (seq_len, hq, hkv, d)
        ctx.save_for_backward(x2, w, cos, sin)
        return kernels().gemm_qkv_rope_w4(x2, w, cos, sin, seq_len, hq, hkv, d)

    @staticmethod
    def backward(ctx, dq):
        x2, w, cos, sin = ctx.saved_tensors
        seq_len, hq, hkv, d = ctx.cfg
        dq = dq.contiguous()
        dw = Fx.weight_grad_async(dq, x2, ctx.sink)
        dx = Fx.mm_dx(dq, w)
        return dx, dw, None, None, None, None, None, None, None


def qkv_rope_attention(xn, wqkv, sink, cos, sin, seq_len, hq, hkv, d, keep: Optional[AttentionKeep] = None,
                       gen: int = -1):
    """QKV projection + RoPE + causal GQA attention (reference model.py:179-212). Returns o [.., Hq D]."""
    x2 = xn.reshape(-1, xn.shape[-1])
    if _qkv_rope_ok(x2, wqkv, d):
        qkv = QKVRopeFn.apply(x2.contiguous(), wqkv, sink, cos, sin, seq_len, hq, hkv, d)
        return rope_attention(qkv, cos, sin, seq_len, hq, hkv, d, keep, gen, rotated=True)
    qkv = Fx.linear(xn, wqkv, sink)
    return rope_attention(qkv.view(-1, qkv.shape[-1]), cos, sin, seq_len, hq, hkv, d, keep, gen)


# functional.py re-exports this module's names at its end and this module calls into functional at
# run time: imported last, so either module can be imported first
from . import functional as Fx  # noqa: E402
