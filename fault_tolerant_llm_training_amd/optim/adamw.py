"""Flat-buffer AdamW with on-device gradient clipping.

Replaces the reference's ``torch.optim.AdamW(model.parameters(), lr,
fused=args.fused_optimizer)`` (train.py:68) plus ``clip_grad_norm_``
(utils.py:58-63). Hyper-parameters default to torch AdamW's (betas 0.9/0.999,
eps 1e-8, weight_decay 0.01). It subclasses ``torch.optim.Optimizer`` so
``LambdaLR`` drives its learning rate exactly as in the reference, and its
``state_dict()`` has torch AdamW's structure (per-parameter ``step``,
``exp_avg``, ``exp_avg_sq`` + ``param_groups``) so checkpoints interoperate
with the reference layout.

On the GPU a step is: one multi-block sum-of-squares over the flat gradient
buffer, one finishing block that computes the norm and clip coefficient into a
device tensor, and one streaming AdamW kernel over the flat parameter /
gradient / moment buffers that reads the coefficient from HBM — no host sync.
A non-finite norm makes the kernel skip the update; :meth:`check_finite`
reports it one step later (deferred, so the host never stalls the GPU).
"""
from __future__ import annotations

import math
from typing import Optional

import torch

from .._native import kernels
from ..models.flat import FlatParamSpace


class NonFiniteGradError(RuntimeError):
    pass


class FlatAdamW(torch.optim.Optimizer):
    def __init__(self, params, flat: FlatParamSpace, lr: float = 1e-3, betas=(0.9, 0.999),
                 eps: float = 1e-8, weight_decay: float = 1e-2, state_dtype: Optional[torch.dtype] = None,
                 max_grad_norm: float = 0.0, fused: bool = True):
        params = list(params)
        defaults = dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay, amsgrad=False,
                        maximize=False, foreach=None, capturable=False, differentiable=False,
                        fused=fused, decoupled_weight_decay=True)
        super().__init__(params, defaults)
        self.flat = flat
        sd = state_dtype or flat.dtype
        self.exp_avg = torch.zeros(flat.numel, dtype=sd, device=flat.device)
        self.exp_avg_sq = torch.zeros(flat.numel, dtype=sd, device=flat.device)
        self.step_count = 0
        self.max_grad_norm = float(max_grad_norm)
        self.stats = torch.zeros(3, dtype=torch.float32, device=flat.device)  # norm, coef, nonfinite
        self._host_stats = torch.zeros(3, dtype=torch.float32, pin_memory=flat.device.type == "cuda")
        self._stats_event = None
        self._stats_step = -1
        # parameter index (reference order) -> flat slot
        name_of = {id(p): n for n, p in flat.param_objs.items()}
        self._index_slots = [flat.slots[name_of[id(p)]] for p in params]

    # ------------------------------------------------------------------ step
    @torch.no_grad()
    def clip_grad_norm_(self, max_norm: Optional[float] = None) -> torch.Tensor:
        """Compute ||g|| and the clip coefficient on device; returns the norm (device scalar)."""
        mn = self.max_grad_norm if max_norm is None else float(max_norm)
        self.max_grad_norm = mn
        g = self.flat.grads
        if g.is_cuda:
            kernels().grad_norm_(g, self.stats, mn)
        else:
            norm = torch.linalg.vector_norm(g.float())
            bad = not torch.isfinite(norm)
            coef = 1.0 if (mn <= 0 or bad) else min(1.0, mn / (float(norm) + 1e-6))
            self.stats.copy_(torch.tensor([float(norm), coef, 1.0 if bad else 0.0]))
        self._clipped = True
        return self.stats[0]

    @torch.no_grad()
    def step(self, closure=None):
        if not getattr(self, "_clipped", False):
            self.clip_grad_norm_()
        self._clipped = False
        self.step_count += 1
        grp = self.param_groups[0]
        lr = float(grp["lr"])
        b1, b2 = grp["betas"]
        eps, wd = grp["eps"], grp["weight_decay"]
        f = self.flat
        if f.params.is_cuda:
            kernels().adamw_(f.params, f.grads, self.exp_avg, self.exp_avg_sq, self.stats, lr, b1, b2,
                             eps, wd, self.step_count)
            self._host_stats.copy_(self.stats, non_blocking=True)
            if self._stats_event is None:
                self._stats_event = torch.cuda.Event()
            self._stats_event.record()
            self._stats_step = self.step_count
        else:
            _adamw_reference(f.params, f.grads, self.exp_avg, self.exp_avg_sq, self.stats, lr, b1, b2,
                             eps, wd, self.step_count)
            self._host_stats.copy_(self.stats)
            self._stats_step = self.step_count
        return None

    def check_finite(self, block: bool = False) -> Optional[float]:
        """Deferred non-finite check of the last step's gradient norm.

        Returns the norm when available. Raises :class:`NonFiniteGradError` (the
        reference's ``error_if_nonfinite`` RuntimeError path) if it was not finite.
        """
        if self._stats_step < 0:
            return None
        ev = self._stats_event
        if ev is not None and not block and not ev.query():
            return None
        if ev is not None and block:
            ev.synchronize()
        norm, _coef, bad = self._host_stats.tolist()
        if bad:
            step = self._stats_step
            self._stats_step = -1
            raise NonFiniteGradError(
                f"The total norm of order 2.0 for gradients from `parameters` is non-finite at optimizer step {step}, "
                "so it cannot be clipped (update skipped)."
            )
        return norm

    def zero_grad(self, set_to_none: bool = True):
        """No-op: every backward overwrites the flat gradient buffer (beta=0 writes)."""
        return None

    # ------------------------------------------------------------------ state dict
    def state_dict(self, exp_avg: Optional[torch.Tensor] = None, exp_avg_sq: Optional[torch.Tensor] = None):
        """torch AdamW ``state_dict`` structure; moments are views of the flat buffers
        (or of ``exp_avg``/``exp_avg_sq`` — e.g. their host snapshot — when given)."""
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
        for key, buf in (("exp_avg", self.exp_avg), ("exp_avg_sq", self.exp_avg_sq)):
            tensors = {i: st[i][key] for i in slots_by_idx if i in st}
            src = None
            if len(tensors) == len(slots_by_idx):
                src = _flat_source(tensors, slots_by_idx, buf.numel(), buf.dtype)
            if src is not None:
                buf.copy_(src, non_blocking=True)
                continue
            for i, t in tensors.items():
                s = slots_by_idx[i]
                buf[s.offset : s.offset + s.numel].view(s.shape).copy_(t, non_blocking=True)
        steps = {int(float(st[i]["step"])) for i in slots_by_idx if i in st}
        if steps:
            self.step_count = max(steps)
        for g, sg in zip(self.param_groups, sd["param_groups"]):
            for k, v in sg.items():
                if k != "params":
                    g[k] = v

    def moments(self):
        return self.exp_avg, self.exp_avg_sq


def _adamw_reference(p, g, m, v, stats, lr, b1, b2, eps, wd, step):
    """CPU reference of the fused kernel (fp32 math, storage dtype rounding)."""
    if stats[2].item() != 0:
        return
    coef = stats[1].item()
    gf = g.float() * coef
    pf = p.float() * (1 - lr * wd)
    mf = m.float()
    vf = v.float()
    mf.add_((gf - mf) * (1 - b1))
    vf.mul_(b2).add_((1 - b2) * gf * gf)
    bc1 = 1 - b1 ** step
    bc2 = 1 - b2 ** step
    denom = vf.sqrt() / math.sqrt(bc2) + eps
    pf.sub_((lr / bc1) * mf / denom)
    p.copy_(pf)
    m.copy_(mf)
    v.copy_(vf)
