"""Bit-level fingerprints of the training state, for resume-equivalence checks at full scale.

A Llama-3-8B state is 48 GB per copy; comparing an uninterrupted run with an interrupted-and-resumed
one through checkpoint files needs three of them on disk. Instead each run logs a digest of its
final parameters and AdamW moments (``--state-digest``) and only the interruption's checkpoint is
written. The digest is an order-independent exact integer sum, so it is deterministic on any
device: every element's raw bits (int16 view for 16-bit dtypes, int32 for fp32) times a
position-dependent weight, summed in int64 with wrap-around. Any bit flip or displaced element
changes it; equal states give equal digests.
"""
from __future__ import annotations

import torch

_CHUNK = 1 << 27
_MOD = 1_000_003


def tensor_digest(t: torch.Tensor) -> str:
    """16-hex-digit digest of the raw bits of ``t`` (any shape, contiguous or not)."""
    flat = t.detach().reshape(-1)
    if flat.dtype in (torch.bfloat16, torch.float16):
        bits = flat.view(torch.int16)
    elif flat.dtype == torch.float32:
        bits = flat.view(torch.int32)
    elif flat.dtype == torch.float64:
        bits = flat.view(torch.int64)
    else:
        bits = flat
    total = torch.zeros((), dtype=torch.int64, device=flat.device)
    for lo in range(0, bits.numel(), _CHUNK):
        b = bits[lo : lo + _CHUNK].to(torch.int64)
        w = torch.arange(lo, lo + b.numel(), dtype=torch.int64, device=b.device).remainder_(_MOD).add_(1)
        total += (b * w).sum()
    return f"{int(total.item()) & 0xFFFFFFFFFFFFFFFF:016x}"


def state_digest(params: torch.Tensor, exp_avg: torch.Tensor, exp_avg_sq: torch.Tensor) -> dict:
    return {"params": tensor_digest(params), "exp_avg": tensor_digest(exp_avg),
            "exp_avg_sq": tensor_digest(exp_avg_sq)}
