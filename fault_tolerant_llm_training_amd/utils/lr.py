"""Learning-rate schedule: linear warmup then constant.

Parity: reference ``utils.py:32-56``. The factor is ``(step+1)/(warmup+1)``
for ``step < warmup`` and ``1.0`` afterwards (the reference docstring mentions
linear decay but the code is constant — SURVEY.md §A.11; we keep the code's
behaviour). ``LambdaLR`` calls ``step()`` once at construction, exactly like the
reference, so the scheduler state dict round-trips with it.
"""
from __future__ import annotations

import functools

from torch.optim.lr_scheduler import LambdaLR


def linear_warmup_constant(warmup_steps: int, current_step: int) -> float:
    if current_step < warmup_steps:
        return float((current_step + 1) / (warmup_steps + 1))
    return 1.0


def build_lr_scheduler(optimizer, warmup_steps: int) -> LambdaLR:
    return LambdaLR(optimizer, functools.partial(linear_warmup_constant, warmup_steps))


def rollback_lr_scheduler(sched: LambdaLR, k: int) -> None:
    """Undo the last ``k`` ``sched.step()`` calls (steps whose optimizer update was skipped
    by the non-finite guard and are rolled back by the trainer)."""
    if k <= 0:
        return
    sched.last_epoch -= k
    if hasattr(sched, "_step_count"):
        sched._step_count -= k
    lrs = [base * lam(sched.last_epoch) for base, lam in zip(sched.base_lrs, sched.lr_lambdas)]
    for g, lr in zip(sched.optimizer.param_groups, lrs):
        g["lr"] = lr
    sched._last_lr = lrs
