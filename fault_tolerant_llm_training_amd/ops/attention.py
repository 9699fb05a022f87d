"""Causal GQA flash attention on packed projections (gfx950 HIP kernels).

Inputs are the rotated ``qk`` buffer ``[T, (Hq+Hkv)*D]`` written by the RoPE
kernel and the fused ``qkv`` projection ``[T, (Hq+2Hkv)*D]`` (V is read in
place). KV heads are indexed as ``h // (Hq/Hkv)`` inside the kernel, so the
reference's materialised ``repeat_kv`` (model.py:129-138) and the
transpose/contiguous copies (model.py:207-213) never exist.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

import os

from .._native import kernels

_USE_HIP_FLASH = True
# Backward variant: 1 = deterministic (default): KV-major dK/dV kernel + Q-major dQ
# kernel, no atomics, bit-reproducible — GPU resume is bit-exact with it and it runs
# as fast as 0 = dQ accumulated with fp32 atomics in the KV-major kernel (330 vs 335 us
# on the Llama-3-8B layer shape, profiles/r1_flash_bench.log).
_BWD_MODE = int(os.environ.get("FT_FLASH_BWD_MODE", "1"))


def set_deterministic(flag: bool) -> None:
    global _BWD_MODE
    _BWD_MODE = 1 if flag else 0


def _split(qk, qkv, S, hq, hkv, d):
    T = qk.shape[0]
    B = T // S
    q = qk[:, : hq * d].view(B, S, hq, d).transpose(1, 2)
    k = qk[:, hq * d :].view(B, S, hkv, d).transpose(1, 2)
    v = qkv[:, (hq + hkv) * d :].view(B, S, hkv, d).transpose(1, 2)
    return q, k, v


def _sdpa(qk, qkv, S, hq, hkv, d):
    q, k, v = _split(qk, qkv, S, hq, hkv, d)
    o = F.scaled_dot_product_attention(q, k, v, is_causal=True, enable_gqa=hq != hkv)
    return o.transpose(1, 2).reshape(qk.shape[0], hq * d)


def flash_attn_fwd(qk, qkv, S, hq, hkv, d):
    """Returns (o [T, Hq*D] bf16, lse [B, Hq, S] fp32)."""
    if _USE_HIP_FLASH and hasattr(kernels(), "flash_fwd"):
        return tuple(kernels().flash_fwd(qk, qkv, S, hq, hkv, d))
    with torch.no_grad():
        return _sdpa(qk, qkv, S, hq, hkv, d), torch.empty(0, device=qk.device)


def flash_attn_bwd(do, qk, qkv, o, lse, S, hq, hkv, d):
    """Returns dqkv [T, (Hq+2Hkv)*D] with dQ/dK still in the rotated frame."""
    if _USE_HIP_FLASH and hasattr(kernels(), "flash_bwd"):
        return kernels().flash_bwd(do, qk, qkv, o, lse, S, hq, hkv, d, _BWD_MODE)
    with torch.enable_grad():
        qk_ = qk.detach().requires_grad_(True)
        qkv_ = qkv.detach().requires_grad_(True)
        out = _sdpa(qk_, qkv_, S, hq, hkv, d)
        dqk, dqkv = torch.autograd.grad(out, (qk_, qkv_), do)
    dqkv = dqkv.contiguous()
    dqkv[:, : (hq + hkv) * d] = dqk
    return dqkv
