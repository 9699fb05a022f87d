"""Training state ↔ checkpoint dict (reference keys).

:func:`build_checkpoint` assembles the dict the engine serialises. Its tensors
are views of the host copies of the flat buffers, so the archive holds one
storage per flat buffer and every ``state_dict`` tensor is an offset view
into it — exactly what ``torch.load`` rebuilds.

:func:`restore_model` / :func:`restore_optimizer` accept both our files (fast
path: one H2D copy per flat buffer when the storage layout matches) and any
reference-layout file (per-tensor copies, e.g. written by the reference's
``torch.save``), with ``_orig_mod.`` prefixes stripped and strict key checking
(the reference's ``strict=False`` load silently kept random
weights after ``--compile``).
"""
from __future__ import annotations

import hashlib
from collections import OrderedDict
from dataclasses import asdict
from typing import Any, Dict, Optional

import torch

from .format import FORMAT_TAG, strip_compile_prefix


def layout_hash(model) -> str:
    flat = model.flat
    h = hashlib.sha1()
    for name, s in flat.slots.items():
        h.update(f"{name}:{s.shape}:{s.offset};".encode())
    h.update(str(flat.dtype).encode())
    return h.hexdigest()[:16]


def _view(buf: torch.Tensor, s) -> torch.Tensor:
    return buf[s.offset : s.offset + s.numel].view(s.shape)


def build_checkpoint(model, optimizer, lr_scheduler, training_step: int, host: Dict[str, torch.Tensor],
                     data_loader: Any = None, rng: Optional[Dict[str, Any]] = None,
                     extra_meta: Optional[Dict[str, Any]] = None) -> Dict[str, Any]:
    flat = model.flat
    P = host["params"]
    model_sd = OrderedDict()
    for name in model.state_dict().keys():
        model_sd[name] = _view(P, flat.slots[name])
    opt_sd = optimizer.state_dict(exp_avg=host["exp_avg"], exp_avg_sq=host["exp_avg_sq"])
    meta = {
        "format": FORMAT_TAG,
        "model_args": asdict(model.model_args),
        "layout_hash": layout_hash(model),
        "flat_numel": int(flat.numel),
        "dtype": str(flat.dtype),
    }
    if extra_meta:
        meta.update(extra_meta)
    out = {
        "model": model_sd,
        "optimizer": opt_sd,
        "lr_scheduler": lr_scheduler.state_dict(),
        "training_step": int(training_step),
        "data_loader": data_loader,
        "meta": meta,
    }
    if rng is not None:
        out["rng"] = rng
    return out


def _flat_source(tensors, slots, numel: int, dtype) -> Optional[torch.Tensor]:
    """If every tensor views one storage at its slot offset, return that storage as a flat tensor."""
    base = None
    for name, t in tensors.items():
        s = slots.get(name)
        if s is None or t.dtype != dtype or tuple(t.shape) != tuple(s.shape) or not t.is_contiguous():
            return None
        st = t.untyped_storage()
        if base is None:
            base = st
        elif st.data_ptr() != base.data_ptr():
            return None
        if t.storage_offset() != s.offset:
            return None
    if base is None or base.nbytes() < numel * torch.tensor([], dtype=dtype).element_size():
        return None
    return torch.empty(0, dtype=dtype).set_(base)[:numel]


@torch.no_grad()
def restore_model(model, sd: Dict[str, torch.Tensor]) -> str:
    """Copy a checkpoint ``model`` dict into the flat parameter buffer. Returns the path taken."""
    flat = model.flat
    sd = strip_compile_prefix(sd)
    expected = list(model.state_dict().keys())
    missing = [k for k in expected if k not in sd]
    unexpected = [k for k in sd if k not in flat.slots]
    if missing or unexpected:
        raise KeyError(f"checkpoint/model mismatch: missing={missing[:5]} unexpected={unexpected[:5]}")
    src = _flat_source(sd, flat.slots, flat.numel, flat.dtype)
    if src is not None:
        from .restore import h2d

        h2d(flat.params, src)
        return "flat"
    for name in expected:
        _view(flat.params, flat.slots[name]).copy_(sd[name], non_blocking=True)
    return "per-tensor"


def capture_rng(device: torch.device) -> Dict[str, Any]:
    r = {"torch": torch.get_rng_state()}
    if device.type == "cuda":
        r["cuda"] = torch.cuda.get_rng_state(device)
    return r


def restore_rng(r: Optional[Dict[str, Any]], device: torch.device) -> None:
    if not r:
        return
    if "torch" in r:
        torch.set_rng_state(r["torch"])
    if device.type == "cuda" and "cuda" in r:
        torch.cuda.set_rng_state(r["cuda"], device)


def shard_regions(model, optimizer, rank: int, world: int, align: int = 2048):
    """This rank's pieces of (params, exp_avg, exp_avg_sq) for a sharded save.

    Parameters (replicated): a contiguous 1/W slice, cut at ``align``-element (4 KiB)
    boundaries so every rank's bytes start O_DIRECT-aligned in the file. AdamW moments:
    under ZeRO-1 exactly the shards this rank owns (bucket by bucket); replicated
    otherwise, 1/W slices like the parameters.
    """
    from .engine import Region

    flat = model.flat
    P = flat.numel

    def cut(n):
        bounds = [min(n, (n * i // world) // align * align) for i in range(world)] + [n]
        return bounds[rank], bounds[rank + 1]

    lo, hi = cut(P)
    regions = [Region("params", flat.params[lo:hi], [(lo, 0, hi - lo)], P)]
    if optimizer.zero1:
        pieces = [(flo, slo, n) for flo, slo, n in optimizer.shard_pieces()]
        regions.append(Region("exp_avg", optimizer.exp_avg, pieces, P))
        regions.append(Region("exp_avg_sq", optimizer.exp_avg_sq, pieces, P))
    else:
        for name, buf in (("exp_avg", optimizer.exp_avg), ("exp_avg_sq", optimizer.exp_avg_sq)):
            regions.append(Region(name, buf[lo:hi], [(lo, 0, hi - lo)], P))
    return regions
