"""Whole training steps as one HIP graph (launch-bound presets).

A GPT-2-small step on one MI355X issues ~400 kernels; the host needs 9.5 ms to enqueue
them and the GPU 8.3 ms to run them (scripts/host_overhead.py), so the step is bound by
Python/launch overhead. :class:`GraphedStep` captures

    optimizer(step k)  ‖  forward(k+1) → backward(k+1) (bucket hooks, dW side stream)

as one graph and replays it: the optimizer of the previous step stays overlapped with the
next forward exactly as in eager mode (the per-layer ParamGate waits become graph edges),
and the host only stages the batch and the step's [lr, 1/bc1, 1/sqrt(bc2)] (a device
buffer the AdamW kernel reads in graph mode) before each replay.

Protocol: ``prime(batch)`` runs forward/backward of the first step eagerly and captures;
``step(batch)`` replays (optimizer of the previous step + forward/backward of ``batch``)
and returns the loss tensor; ``finish()`` runs the last pending optimizer step eagerly.
The host-side bookkeeping (optimizer step counter, LR scheduler, non-finite stats ring)
advances per replay as in eager mode. Math is identical to eager (same kernels, same
order): tests/test_graphs_gpu.py checks the parameters bit for bit.
"""
from __future__ import annotations

from typing import Callable, Optional

import torch

import os

from ._native import kernels
from .ops.functional import join_dw_stream


def hw_queue_problem() -> str:
    """Why the whole-step graph must not run under this process's HIP queue setting, or "". With
    GPU_MAX_HW_QUEUES=2 the HIP runtime segfaults inside hipGraphLaunch on the replay of this
    multi-stream graph (GPT-2-small, profiles/r6/hw_queues_ab.log); 8 queues replay 2.7x slower."""
    q = os.environ.get("GPU_MAX_HW_QUEUES")
    if q is not None and q.strip().isdigit() and int(q) < 4:
        return (f"GPU_MAX_HW_QUEUES={q}: the HIP runtime crashes replaying the multi-stream step graph "
                "with fewer than 4 hardware queues (leave it at the default 4)")
    return ""


class GraphedStep:
    def __init__(self, model, reducer, optimizer, lr_scheduler,
                 fwd_bwd: Callable[[torch.Tensor, torch.Tensor], torch.Tensor]):
        self.model, self.red, self.opt, self.sched = model, reducer, optimizer, lr_scheduler
        self.fwd_bwd = fwd_bwd
        self.graph: Optional[torch.cuda.CUDAGraph] = None
        self.tok: Optional[torch.Tensor] = None
        self.lab: Optional[torch.Tensor] = None
        self.loss: Optional[torch.Tensor] = None
        self.pending = False  # a backward whose optimizer step has not run yet
        self.cap_stream: Optional[torch.cuda.Stream] = None
        # data parallel: every collective of the step on the reducer's side stream (the form RCCL
        # collectives capture in: ddp.GradReducer.single_stream)
        reducer.single_stream = bool(reducer.comm)

    def _join(self) -> None:
        cur = torch.cuda.current_stream()
        join_dw_stream()
        if self.red.side is not None:
            cur.wait_stream(self.red.side)


    def _opt_step(self) -> None:
        self.opt.clip_grad_norm_(self.opt.max_grad_norm)
        self.opt.step()

    @property
    def ready(self) -> bool:
        """A captured graph and a pending backward: the next step can be a replay."""
        return self.graph is not None and self.pending

    def prime(self, tok: torch.Tensor, lab: torch.Tensor) -> torch.Tensor:
        """Eager forward/backward of this step, then capture (nothing runs during capture).
        Called again after :meth:`finish` (e.g. around a checkpoint) to re-enter graph mode."""
        self.graph = None  # release a previous capture's pool first
        self.tok = torch.empty_like(tok, device=self.model.flat.device)
        self.lab = torch.empty_like(lab, device=self.model.flat.device)
        self.tok.copy_(tok, non_blocking=True)
        self.lab.copy_(lab, non_blocking=True)
        loss = self.fwd_bwd(self.tok, self.lab)
        self._join()
        self.pending = True
        torch.cuda.synchronize()
        self.opt.graph_mode = True
        g = torch.cuda.CUDAGraph()
        sc0 = self.opt.step_count
        if self.cap_stream is None:
            # one capture stream per GraphedStep, with its own split-K hand-off flags (allocated
            # here: nothing can be allocated during capture), so the captured split products keep
            # the eager step's summation order and never share flags with an eager launch
            self.cap_stream = torch.cuda.Stream()
            with torch.cuda.stream(self.cap_stream):
                kernels().gemm_w4_prepare_capture()
        # thread-local capture: in the default global mode any HIP call another thread makes while
        # the capture is open fails -- the RCCL watchdog thread polling the events of earlier
        # (already finished) collectives then got hipErrorCapturedEvent and took the process down
        # (1 run in ~7 of the DP graph test, even with TORCH_NCCL_RETHROW_CUDA_ERRORS=0); only the
        # capturing thread's own calls need the check
        with torch.cuda.graph(g, stream=self.cap_stream, capture_error_mode="thread_local"):
            self._opt_step()  # (its host-side step count is reset below; hyper is read on device)
            self.loss = self.fwd_bwd(self.tok, self.lab)
            self._join()
        self.opt.step_count = sc0
        self.opt.gate.entries.clear()  # their waits are edges inside the graph now
        self.graph = g
        return loss

    def step(self, tok: torch.Tensor, lab: torch.Tensor) -> torch.Tensor:
        """Optimizer step of the pending backward + forward/backward of (tok, lab)."""
        assert self.graph is not None and self.pending
        self.opt.step_count += 1
        self.opt.stage_hyper(self.opt.step_count)
        self.tok.copy_(tok, non_blocking=True)
        self.lab.copy_(lab, non_blocking=True)
        self.graph.replay()
        self.opt.publish_stats()
        self.sched.step()
        return self.loss

    def finish(self) -> None:
        """Run the pending optimizer step eagerly (same kernels, device hyperparameters)."""
        if not self.pending:
            return
        self.opt.step_count += 1
        self.opt.stage_hyper(self.opt.step_count)
        self.opt.step_count -= 1  # step() increments it again
        self._opt_step()
        # the norm / non-finite flag were written on the optimizer (side) stream; the host copy below
        # runs on this stream: without the join it could read the previous step's stats (a poisoned
        # step then looked finite and was not rolled back -- a race seen once on the GPU suite)
        self._join()
        self.opt.publish_stats()
        self.sched.step()
        self.pending = False
