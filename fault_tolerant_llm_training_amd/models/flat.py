"""Flat parameter / gradient storage.

All parameters of a model live in ONE contiguous device buffer and all their
gradients in a second buffer with the identical layout. Each ``nn.Parameter``
is a view into the parameter buffer and its ``.grad`` a view into the gradient
buffer, so:

* fused projections are free: ``wq|wk|wv`` and ``w1|w3`` are laid out
  back-to-back, so the concatenated weight of one fused GEMM is just a view;
* the optimizer, the gradient-norm reduction and the checkpoint snapshot each
  work on a handful of huge contiguous ranges (one kernel / one DMA each);
* data-parallel buckets are contiguous ranges of the gradient buffer.

The layout order is chosen for these uses; the ``nn.Module`` registration order
(and therefore ``state_dict`` keys and optimizer parameter indices) stays
identical to the reference (model.py:257-352).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, List, Sequence, Tuple

import torch
import torch.nn as nn

from ..ops.grad_sink import GradSink

ALIGN = 64  # elements (128 B for bf16): every param starts 16-B aligned for vector access


@dataclass
class Slot:
    name: str
    shape: Tuple[int, ...]
    offset: int
    numel: int


class FlatParamSpace:
    def __init__(self, model: nn.Module, layout: Sequence[str], device, dtype: torch.dtype):
        named = dict(model.named_parameters())
        missing = set(named) - set(layout)
        extra = set(layout) - set(named)
        if missing or extra:
            raise ValueError(f"flat layout mismatch: missing={sorted(missing)} extra={sorted(extra)}")
        self.device = torch.device(device)
        self.dtype = dtype
        self.slots: Dict[str, Slot] = {}
        off = 0
        for name in layout:
            p = named[name]
            n = p.numel()
            self.slots[name] = Slot(name, tuple(p.shape), off, n)
            off += (n + ALIGN - 1) // ALIGN * ALIGN
        # a multiple of ALIGN: every bucket cut at slot boundaries splits evenly into
        # 8-element-aligned ZeRO shards for up to 8 ranks
        self.numel = (off + ALIGN - 1) // ALIGN * ALIGN
        self.align = ALIGN
        self.params = torch.zeros(self.numel, dtype=dtype, device=self.device)
        # zero-initialised once: alignment gaps stay zero forever (no NaN in the norm)
        self.grads = torch.zeros(self.numel, dtype=dtype, device=self.device)
        self.layout = list(layout)
        self.model_ref = None
        self.sinks: Dict[str, GradSink] = {}
        self.param_objs: Dict[str, nn.Parameter] = {}
        modules = dict(model.named_modules())
        for name in layout:
            s = self.slots[name]
            mod_name, _, attr = name.rpartition(".")
            mod = modules[mod_name]
            pv = self.params[s.offset : s.offset + s.numel].view(s.shape)
            gv = self.grads[s.offset : s.offset + s.numel].view(s.shape)
            newp = nn.Parameter(pv, requires_grad=True)
            newp.grad = gv
            sink = GradSink(gv, s.offset, s.offset + s.numel, name)
            newp._ft_sink = sink
            self.sinks[name] = sink
            self.param_objs[name] = newp
            setattr(mod, attr, newp)

    # ---------------------------------------------------------------- fused views
    def fused(self, names: List[str]) -> Tuple[torch.Tensor, GradSink]:
        """Concatenation (along dim 0) of adjacent 2-D params as one weight view + sink."""
        slots = [self.slots[n] for n in names]
        for a, b in zip(slots, slots[1:]):
            if a.offset + a.numel != b.offset:
                raise ValueError(f"params {a.name} and {b.name} are not adjacent in the flat buffer")
            if a.shape[1:] != b.shape[1:]:
                raise ValueError("fused params must share trailing dims")
        start = slots[0].offset
        end = slots[-1].offset + slots[-1].numel
        rows = sum(s.shape[0] for s in slots)
        shape = (rows,) + tuple(slots[0].shape[1:])
        w = self.params[start:end].view(shape)
        g = self.grads[start:end].view(shape)
        return w, GradSink(g, start, end, "+".join(names))

    def ranges(self) -> List[Tuple[str, int, int]]:
        return [(n, s.offset, s.offset + s.numel) for n, s in self.slots.items()]

    def nbytes(self) -> int:
        return self.params.numel() * self.params.element_size()
