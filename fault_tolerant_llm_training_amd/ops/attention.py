"""Causal GQA flash attention on packed projections (gfx950 HIP kernels).

Q and K come rotated (reference model.py:100-126) from one of two producers:
by default the QKV projection's GEMM epilogue (``gemm_qkv_rope_w4``, csrc/kernels/gemm_w4.hip)
rotates them in place, so ``qk`` IS the packed ``qkv`` projection ``[T, (Hq+2Hkv)*D]``; on the
paths without that epilogue (fp32, GPT-2-sized models, FT_QKV_ROPE=0) the RoPE kernel
(csrc/kernels/rope.hip) writes a separate rotated ``qk`` buffer ``[T, (Hq+Hkv)*D]``. V is always
read in place from ``qkv``. KV heads are indexed as ``h // (Hq/Hkv)`` inside the kernels, so
the reference's materialised ``repeat_kv`` (model.py:129-138) and the transpose/contiguous
copies (model.py:207-213) never exist. This module picks the kernel family by dtype
(bf16/fp16: csrc/kernels/flash_attn.hip, fp32: csrc/kernels/flash_f32.hip) and exposes the
deterministic / non-deterministic backward switch.
"""
from __future__ import annotations

import os

import torch

from .._native import kernels

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
