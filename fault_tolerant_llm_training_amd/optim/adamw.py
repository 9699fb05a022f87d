"""Flat-buffer AdamW with on-device gradient clipping, pipelined into the next step.

Replaces the reference's ``torch.optim.AdamW(model.parameters(), lr,
fused=args.fused_optimizer)`` (train.py:68) plus ``clip_grad_norm_``
(utils.py:58-63). Hyper-parameters default to torch AdamW's (betas 0.9/0.999,
eps 1e-8, weight_decay 0.01). It subclasses ``torch.optim.Optimizer`` so
``LambdaLR`` drives its learning rate exactly as in the reference, and its
``state_dict()`` has torch AdamW's structure (per-parameter ``step``,
``exp_avg``, ``exp_avg_sq`` + ``param_groups``) so checkpoints interoperate
with the reference layout.

GPU step (with a :class:`~..parallel.ddp.GradReducer`):

1. the reducer already summed squares of every gradient bucket on a side
   stream while backward was running (after its all-reduce / reduce-scatter);
2. ``step()`` enqueues on that side stream: the norm + clip coefficient
   (one block; ZeRO-1 adds a 4-byte all-reduce), then one AdamW launch per
   bucket **in forward order** (embedding first), each followed by an event
   (or, under ZeRO-1, the bucket's parameter all-gather);
3. the next forward waits, layer by layer, only for the buckets holding that
   layer's weights (:class:`ParamGate`), so the bandwidth-bound optimizer pass
   overlaps the compute-bound GEMMs of the next step instead of running as a
   serial phase.

A non-finite norm makes every update kernel skip (no host sync), and the flag is
*sticky*: every later step skips too until :meth:`reset_nonfinite`. The host
reads each step's ``[norm, coef, nonfinite]`` from a small ring of pinned
copies; the trainer checks step ``k`` at the boundary before step ``k+2``
(that copy has long landed, so the check never stalls the pipeline) and, on a
bad step, rolls the host counters back to it with :meth:`rollback_steps`:
parameters and moments are still exactly those before the bad step, which is
what the reference's ``error_if_nonfinite`` raise before ``optimizer.step()``
leaves behind (reference utils.py:61, train.py:107-109).
"""
from __future__ import annotations

import math
from typing import List, Optional, Tuple

import torch
import torch.distributed as dist

from .._native import kernels, native
from ..models.flat import FlatParamSpace


class NonFiniteGradError(RuntimeError):
    pass


class ParamGate:
    """Per-range readiness of the parameter buffer for the next forward.

    Entries are (lo, hi, handle) with handle a ``torch.cuda.Event`` (recorded on
    the optimizer stream) or a collective work object (all-gather). The model
    calls :meth:`wait` with the flat range of the weights it is about to use;
    the *compute stream* is made to wait — the host never blocks.
    """

    def __init__(self):
        self.entries: List[list] = []

    def add(self, lo: int, hi: int, handle) -> None:
        self.entries.append([lo, hi, handle])

    def wait(self, lo: int, hi: int) -> None:
        if not self.entries:
            return
        cur = None
        for e in self.entries:
            h = e[2]
            if h is None or e[1] <= lo or e[0] >= hi:
                continue
            if isinstance(h, torch.cuda.Event):
                if cur is None:
                    cur = torch.cuda.current_stream()
                cur.wait_event(h)
            else:
                h.wait()
            e[2] = None
        self.entries = [e for e in self.entries if e[2] is not None]

    def wait_all(self) -> None:
        if self.entries:
            self.wait(0, 1 << 62)


class FlatAdamW(torch.optim.Optimizer):
    RING = 4  # pinned stats copies kept (the trainer checks two steps late)

    def __init__(self, params, flat: FlatParamSpace, lr: float = 1e-3, betas=(0.9, 0.999),
                 eps: float = 1e-8, weight_decay: float = 1e-2, state_dtype: Optional[torch.dtype] = None,
                 max_grad_norm: float = 0.0, fused: bool = True, reducer=None):
        params = list(params)
        defaults = dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay, amsgrad=False,
                        maximize=False, foreach=None, capturable=False, differentiable=False,
                        fused=fused, decoupled_weight_decay=True)
        super().__init__(params, defaults)
        self.flat = flat
        self.reducer = reducer
        self.zero1 = reducer is not None and reducer.mode == "zero1"
        sd = state_dtype or flat.dtype
        n = reducer.shard_numel if self.zero1 else flat.numel
        self.exp_avg = torch.zeros(n, dtype=sd, device=flat.device)
        self.exp_avg_sq = torch.zeros(n, dtype=sd, device=flat.device)
        self.step_count = 0
        self.max_grad_norm = float(max_grad_norm)
        self.stats = torch.zeros(3, dtype=torch.float32, device=flat.device)  # norm, coef, nonfinite
        # ring of per-step host copies: step -> (pinned [3] copy, event or None)
        self._pin = flat.device.type == "cuda"
        self._ring = [torch.zeros(3, dtype=torch.float32, pin_memory=self._pin) for _ in range(self.RING)]
        self._ring_events = [None] * self.RING
        self._ring_steps = [-1] * self.RING
        self._checked_step = 0  # every step <= this one is known finite
        self._stats_event = None
        self._stats_step = -1
        self.gate = ParamGate()
        # HIP-graph mode (graphs.GraphedStep): lr and bias corrections come from this device
        # buffer, filled from a ring of pinned host slots before each replay
        self.graph_mode = False
        self.hyper = torch.zeros(3, dtype=torch.float32, device=flat.device)
        self._hyper_ring = [torch.zeros(3, dtype=torch.float32, pin_memory=self._pin) for _ in range(16)]
        self._hyper_i = 0
        # grid cap for the per-bucket AdamW launches that run concurrently with the next
        # forward's GEMMs (fewer blocks = less contention for CU issue slots)
        self.overlap_blocks = 0  # grid cap of the pipelined per-bucket launches (A/B: r2_adamw_overlap_cap.log)
        # parameter index (reference order) -> flat slot
        name_of = {id(p): n for n, p in flat.param_objs.items()}
        self._index_slots = [flat.slots[name_of[id(p)]] for p in params]

    # ------------------------------------------------------------------ step
    def clip_grad_norm_(self, max_norm: Optional[float] = None) -> torch.Tensor:
        """Set the clipping threshold; the norm itself is computed on device by :meth:`step`
        (``stats[0]`` holds it afterwards). Clipping is real."""
        if max_norm is not None:
            self.max_grad_norm = float(max_norm)
        return self.stats[0]

    def _stream_ctx(self):
        r = self.reducer
        if r is not None and r.overlap:
            return torch.cuda.stream(r.side)
        import contextlib

        return contextlib.nullcontext()

    def _hyper(self):
        grp = self.param_groups[0]
        b1, b2 = grp["betas"]
        return float(grp["lr"]), b1, b2, grp["eps"], grp["weight_decay"]

    def stage_hyper(self, step: int) -> None:
        """Graph mode: enqueue the H2D copy of [lr, 1/bc1, 1/sqrt(bc2)] of optimizer step
        ``step`` into ``self.hyper`` (on the current stream, ahead of the replay that uses it),
        rounded to fp32 exactly like the host path of adamw_ (optim.hip): bc = 1.f - (float)beta^step,
        then 1/bc and 1/sqrtf(bc) in float."""
        import numpy as np

        lr, b1, b2, _eps, _wd = self._hyper()
        bc1 = np.float32(1.0) - np.float32(b1 ** step)  # 1.f - (float)std::pow(beta, step)
        bc2 = np.float32(1.0) - np.float32(b2 ** step)
        h = self._hyper_ring[self._hyper_i % len(self._hyper_ring)]
        self._hyper_i += 1
        h.copy_(torch.from_numpy(np.array([np.float32(lr), np.float32(1.0) / bc1,
                                           np.float32(1.0) / np.sqrt(bc2)], dtype=np.float32)))
        self.hyper.copy_(h, non_blocking=True)

    def _update(self, p, g, m, v, lr, b1, b2, eps, wd, max_blocks: int = 0):
        if native(p):
            kernels().adamw_(p, g, m, v, self.stats, lr, b1, b2, eps, wd, self.step_count, max_blocks,
                             self.hyper if self.graph_mode else None)
        else:
            _adamw_reference(p, g, m, v, self.stats, lr, b1, b2, eps, wd, self.step_count)

    @torch.no_grad()
    def step(self, closure=None):
        self.step_count += 1
        lr, b1, b2, eps, wd = self._hyper()
        f = self.flat
        r = self.reducer
        cuda = f.params.is_cuda
        if r is None:
            # stand-alone: whole-buffer norm + one AdamW launch on the current stream
            if cuda:
                from ..ops.functional import join_dw_stream

                join_dw_stream()
            if native(f.grads):
                kernels().grad_norm_(f.grads, self.stats, self.max_grad_norm)
            else:
                gd = f.grads.double() if f.grads.dtype == torch.float64 else f.grads.float()
                _norm_reference(gd.pow(2).sum().reshape(1), self.stats, self.max_grad_norm)
            self._update(f.params, f.grads, self.exp_avg, self.exp_avg_sq, lr, b1, b2, eps, wd)
            self._publish_stats()
            return None
        if r.overlap:
            r.side.wait_stream(torch.cuda.current_stream())
        with self._stream_ctx():
            total = r.global_sumsq()
            if cuda:
                kernels().norm_finish_(total, self.stats, self.max_grad_norm)
            else:
                _norm_reference(total.sum().reshape(1), self.stats, self.max_grad_norm)
            if not self.graph_mode:  # graph replays publish after the replay (publish_stats)
                self._publish_stats()
            for b in sorted(r.buckets, key=lambda b: b.lo):  # forward order
                slo, shi = r.state_range(b)
                self._update(r.param_for_update(b), r.grad_for_update(b), self.exp_avg[slo:shi],
                             self.exp_avg_sq[slo:shi], lr, b1, b2, eps, wd,
                             self.overlap_blocks if r.overlap else 0)
                if self.zero1 and r.dry_comm:
                    pass
                elif self.zero1 and r.single_stream and r.overlap:
                    # whole-step graph: the all-gather blocking on this (side) stream, right behind
                    # the bucket's update (ddp.GradReducer.single_stream); the next forward waits
                    # for its event
                    dist.all_gather_into_tensor(f.params[b.lo : b.hi], r.param_shard(b), group=r.group)
                    b.agevent.record()
                    self.gate.add(b.lo, b.hi, b.agevent)
                elif self.zero1:
                    work = dist.all_gather_into_tensor(f.params[b.lo : b.hi], r.param_shard(b),
                                                       group=r.group, async_op=True)
                    if r.overlap:
                        self.gate.add(b.lo, b.hi, work)
                    else:
                        work.wait()
                elif r.overlap:
                    b.event.record()
                    self.gate.add(b.lo, b.hi, b.event)
        return None

    def _publish_stats(self):
        i = self.step_count % self.RING
        h = self._ring[i]
        if self.stats.is_cuda:
            h.copy_(self.stats, non_blocking=True)
            ev = self._ring_events[i]
            if ev is None:
                ev = self._ring_events[i] = torch.cuda.Event()
            ev.record()
            self._stats_event = ev
        else:
            h.copy_(self.stats)
        self._ring_steps[i] = self.step_count
        self._stats_step = self.step_count

    def publish_stats(self) -> None:
        """Graph mode: copy the stats of the step the last replay ran to the host ring."""
        self._publish_stats()

    def norm_for_logging(self):
        """(device tensor holding the last step's pre-clip grad norm, event after which it is valid)."""
        return self.stats[:1], self._stats_event

    def _step_stats(self, step: int, block: bool):
        """Host copy [norm, coef, nonfinite] of optimizer step ``step`` (None if not ready / gone)."""
        i = step % self.RING
        if self._ring_steps[i] != step:
            return None
        ev = self._ring_events[i]
        if ev is not None:
            if block:
                ev.synchronize()
            elif not ev.query():
                return None
        return self._ring[i].tolist()

    def first_nonfinite(self, upto: Optional[int] = None, block: bool = True) -> Optional[int]:
        """Oldest optimizer step in ``(checked, upto]`` whose gradient norm was not finite.

        ``upto`` defaults to the last step taken. The flag is sticky, so step ``upto``
        alone tells whether any step before it was bad; only then is the ring scanned for
        the first bad one (where the state stopped changing). Steps found finite are never
        read again. A non-blocking call returns None while step ``upto``'s copy is in flight."""
        upto = self.step_count if upto is None else min(int(upto), self.step_count)
        if upto <= self._checked_step:
            return None
        st = self._step_stats(upto, block)
        if st is None:
            return None
        if not st[2]:
            self._checked_step = upto
            return None
        for k in range(max(self._checked_step + 1, self.step_count - self.RING + 1), upto):
            sk = self._step_stats(k, True)
            if sk is not None and sk[2]:
                return k
        return upto

    def last_norm(self) -> Optional[float]:
        st = self._step_stats(self.step_count, True) if self.step_count > 0 else None
        return None if st is None else st[0]

    def check_finite(self, block: bool = False) -> Optional[float]:
        """Non-finite check of every step so far (stand-alone use: bench, smoke, tests).

        Returns the last step's norm when available. Raises :class:`NonFiniteGradError` (the
        reference's ``error_if_nonfinite`` RuntimeError path) if some step was not finite.
        """
        if self.step_count == 0:
            return None
        bad = self.first_nonfinite(block=block)
        if bad is not None:
            raise NonFiniteGradError(nonfinite_message(bad))
        st = self._step_stats(self.step_count, block)
        return None if st is None else st[0]

    @torch.no_grad()
    def reset_nonfinite(self) -> None:
        """Clear the sticky skip flag (after the state was restored from a checkpoint)."""
        self.stats.zero_()
        self._checked_step = self.step_count

    def rollback_steps(self, k: int) -> None:
        """Undo the host-side bookkeeping of the last ``k`` optimizer steps, whose updates the
        (sticky) non-finite guard skipped on device: step counter and stats ring only."""
        if k <= 0:
            return
        self.step_count -= k
        self._checked_step = min(self._checked_step, self.step_count)
        for i in range(self.RING):
            if self._ring_steps[i] > self.step_count:
                self._ring_steps[i] = -1

    def zero_grad(self, set_to_none: bool = True):
        """No-op: every backward overwrites the flat gradient buffer (beta=0 writes)."""
        return None

    # ------------------------------------------------------------------ full-layout state
    def shard_pieces(self) -> List[Tuple[int, int, int]]:
        """ZeRO-1: (flat_lo, state_lo, length) pieces of the full moment layout owned here."""
        r = self.reducer
        return [(b.lo + r.rank * b.shard_len, b.shard_lo, b.shard_len) for b in r.buckets]

    @torch.no_grad()
    def gather_full_state(self, out_m: torch.Tensor, out_v: torch.Tensor) -> None:
        """ZeRO-1: assemble the full-layout moments (flat parameter layout) on every rank."""
        r = self.reducer
        for b in r.buckets:
            slo, shi = r.state_range(b)
            dist.all_gather_into_tensor(out_m[b.lo : b.hi], self.exp_avg[slo:shi], group=r.group)
            dist.all_gather_into_tensor(out_v[b.lo : b.hi], self.exp_avg_sq[slo:shi], group=r.group)

    # ------------------------------------------------------------------ state dict
    def state_dict(self, exp_avg: Optional[torch.Tensor] = None, exp_avg_sq: Optional[torch.Tensor] = None):
        """torch AdamW ``state_dict`` structure; moments are views of full-layout buffers
        (``exp_avg``/``exp_avg_sq`` when given — e.g. their host snapshot — else our own;
        under ZeRO-1 the full layout must be given, see :meth:`gather_full_state`)."""
        if self.zero1 and exp_avg is None:
            raise RuntimeError("ZeRO-1 optimizer state is sharded: pass full-layout moments")
        M = self.exp_avg if exp_avg is None else exp_avg
        V = self.exp_avg_sq if exp_avg_sq is None else exp_avg_sq
        state = {}
        for i, s in enumerate(self._index_slots):
            state[i] = {
                "step": torch.tensor(float(self.step_count), dtype=torch.float32),
                "exp_avg": M[s.offset : s.offset + s.numel].view(s.shape),
                "exp_avg_sq": V[s.offset : s.offset + s.numel].view(s.shape),
            }
        groups = []
        idx = 0
        for g in self.param_groups:
            gg = {k: v for k, v in g.items() if k != "params"}
            gg["params"] = list(range(idx, idx + len(g["params"])))
            idx += len(g["params"])
            groups.append(gg)
        return {"state": state, "param_groups": groups}

    @torch.no_grad()
    def load_state_dict(self, sd):
        """Accepts our files and torch AdamW files (per-parameter tensors) alike."""
        from ..ckpt.state import _flat_source

        st = sd["state"]
        slots_by_idx = {i: s for i, s in enumerate(self._index_slots)}
        numel = self.flat.numel
        for key, buf in (("exp_avg", self.exp_avg), ("exp_avg_sq", self.exp_avg_sq)):
            tensors = {i: st[i][key] for i in slots_by_idx if i in st}
            src = None
            if len(tensors) == len(slots_by_idx):
                src = _flat_source(tensors, slots_by_idx, numel, buf.dtype)
            if src is None:
                # per-tensor file: assemble the full layout on the host first
                src = torch.zeros(numel, dtype=buf.dtype)
                for i, t in tensors.items():
                    s = slots_by_idx[i]
                    src[s.offset : s.offset + s.numel].view(s.shape).copy_(t)
            from ..ckpt.restore import h2d

            if self.zero1:
                for flo, slo, n in self.shard_pieces():
                    h2d(buf[slo : slo + n], src[flo : flo + n])
            else:
                h2d(buf, src)
        steps = {int(float(st[i]["step"])) for i in slots_by_idx if i in st}
        if steps:
            self.step_count = max(steps)
        for g, sg in zip(self.param_groups, sd["param_groups"]):
            for k, v in sg.items():
                if k != "params":
                    g[k] = v

    def moments(self):
        return self.exp_avg, self.exp_avg_sq


def nonfinite_message(step: int) -> str:
    return (f"The total norm of order 2.0 for gradients from `parameters` is non-finite at optimizer step {step}, "
            "so it cannot be clipped (update skipped).")


def _norm_reference(sumsq: torch.Tensor, stats: torch.Tensor, max_norm: float) -> None:
    norm = float(sumsq.sqrt())
    bad = not math.isfinite(norm)
    coef = 1.0 if (max_norm <= 0 or bad) else min(1.0, max_norm / (norm + 1e-6))
    sticky = bad or float(stats[2]) != 0.0  # same sticky flag as norm_finish_kernel
    stats.copy_(torch.tensor([norm, coef, 1.0 if sticky else 0.0]))


def _adamw_reference(p, g, m, v, stats, lr, b1, b2, eps, wd, step):
    """Reference of the fused kernel (fp32 math, storage dtype rounding); fp64 parameters (the
    composed path of --model-dtype fp64) are updated in fp64, as the reference's torch AdamW does."""
    if stats[2].item() != 0:
        return
    coef = stats[1].item()
    md = torch.float64 if p.dtype == torch.float64 else torch.float32
    gf = g.to(md) * coef
    pf = p.to(md) * (1 - lr * wd)
    mf = m.to(md)
    vf = v.to(md)
    mf.add_((gf - mf) * (1 - b1))
    vf.mul_(b2).add_((1 - b2) * gf * gf)
    bc1 = 1 - b1 ** step
    bc2 = 1 - b2 ** step
    denom = vf.sqrt() / math.sqrt(bc2) + eps
    pf.sub_((lr / bc1) * mf / denom)
    p.copy_(pf)
    m.copy_(mf)
    v.copy_(vf)
