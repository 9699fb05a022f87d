"""Gradient sinks: weight gradients are written straight into the flat gradient buffer.

Every parameter (and every fused weight view such as ``[wq; wk; wv]``) owns a
:class:`GradSink` whose ``buf`` is a view into the model-wide flat gradient
buffer. Backward kernels/GEMMs write the weight gradient directly into it
(``beta = 0`` GEMM output, no ``AccumulateGrad`` read-modify-write), then call
:meth:`GradSink.ready` so the data-parallel engine can launch the all-reduce of
any bucket that just became complete while backward keeps running.
"""
from __future__ import annotations

from typing import Callable, Optional

import torch


class GradSink:
    __slots__ = ("buf", "start", "end", "accumulate", "hook", "name", "gather", "defer", "stash", "part", "sq_done")

    def __init__(self, buf: torch.Tensor, start: int = 0, end: int = 0, name: str = ""):
        self.buf = buf
        self.start = start  # element range in the flat buffer
        self.end = end
        self.accumulate = False  # True for micro-batches after the first (grad accumulation)
        self.hook: Optional[Callable[["GradSink"], None]] = None
        self.name = name
        # data parallel: (tokens, dy) -> every rank's (tokens, dy) (sparse embedding exchange)
        self.gather: Optional[Callable] = None
        # gradient accumulation with the sparse exchange: rows of non-final micro-batches are
        # stashed here (defer=True) and exchanged together in the last micro-batch
        self.defer = False
        self.stash: list = []
        # gradient-norm partials (one GPU, parallel.ddp.GradReducer "local" mode): a slice of the
        # reducer's partial sums of squares that the producing kernel fills in its epilogue (the
        # w4 dW GEMM per output tile, the norm backward per column block); it then sets sq_done
        # and the reducer skips the separate sum-of-squares pass over this gradient
        self.part: Optional[torch.Tensor] = None
        self.sq_done = False

    def ready(self) -> None:
        if self.hook is not None:
            self.hook(self)

    # dW = a @ b (written or accumulated into buf)
    def mm(self, a: torch.Tensor, b: torch.Tensor) -> None:
        out = self.buf.view(a.shape[0], b.shape[1])
        if self.accumulate:
            out.addmm_(a, b)
        else:
            torch.mm(a, b, out=out)
        self.ready()

    def set_(self, g: torch.Tensor) -> None:
        if self.accumulate:
            self.buf.add_(g.view_as(self.buf))
        else:
            self.buf.copy_(g.view_as(self.buf))
        self.ready()


def sink_of(p: torch.Tensor) -> Optional[GradSink]:
    return getattr(p, "_ft_sink", None)
