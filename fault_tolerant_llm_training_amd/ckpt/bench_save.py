"""Checkpoint-save measurements for ``bench.py`` (second half of the BASELINE metric).

The reference saves with a synchronous ``torch.save`` at exit: 33.55 s for the
48.3 GB Llama-3-8B state (reference utils.py:74-80). Two numbers
are measured here, both through the same engine the trainer uses
(``ckpt.engine``; sharded over the ranks under data parallelism):

* ``exit_save_s`` — the exit-path save (SIGUSR1 / error): ``save(blocking=True)``
  from call to file durable (fsync + atomic rename). This is what the
  reference's 33.55 s measures; ``vs_baseline_save`` = 33.55 / it.
* ``loaded`` — a periodic (``--save-every``) save while training continues:
  per-step GPU times (events on the compute stream) of steady steps, then of
  every step from the save call until the file is durable. The excess of those
  steps over the steady median is the save's *training-visible* cost
  (``visible_s``): snapshot enqueue on the host, the compute stream's wait for
  the HBM snapshot before the next optimizer step, and the snapshot/drain DMA
  contending with the GEMMs for HBM.

Under data parallelism every step runs collectives, so every rank must run the
same number of steps: the "file durable" test that ends the loaded phase is a
rank-local poll, agreed on after each step over the gloo control group (the save
counts as done once every rank's share is durable). On the CPU (gloo tests) the
step times are host clock stamps after each step instead of device events.
"""
from __future__ import annotations

import os
import statistics
import time

import torch

from .engine import CheckpointEngine
from .format import checkpoint_file
from .state import build_checkpoint, shard_regions


def _engine(model, optimizer, info, mode: str) -> CheckpointEngine:
    if info.world_size > 1:
        return CheckpointEngine(shard_regions(model, optimizer, info.rank, info.world_size), mode=mode,
                                group=info.ckpt_group, rank=info.rank, world=info.world_size, sharded=True)
    return CheckpointEngine({"params": model.flat.params, "exp_avg": optimizer.exp_avg,
                             "exp_avg_sq": optimizer.exp_avg_sq}, mode=mode)


def measure_checkpoint(model, optimizer, lr_scheduler, step_fn, first_step: int, ckpt_dir: str, info,
                       mode: str = "auto", steady_steps: int = 6, max_loaded_steps: int = 400):
    """``step_fn(i, before_opt)`` runs training step ``i`` and calls ``before_opt()`` right before
    the optimizer step. Returns a dict (every rank; rank 0's is reported)."""
    from ..parallel import dist as fdist

    dev = model.flat.device
    cuda = dev.type == "cuda"

    def sync():
        if cuda:
            torch.cuda.synchronize(dev)

    eng = _engine(model, optimizer, info, mode)
    t0 = time.perf_counter()
    eng.preallocate()
    alloc_s = time.perf_counter() - t0
    path = checkpoint_file(ckpt_dir, "bench")

    def build(host):
        return build_checkpoint(model, optimizer, lr_scheduler, 0, host)

    # ---- exit-path save: the training loop is stopped until the file is durable
    optimizer.gate.wait_all()
    sync()
    fdist.barrier()
    t0 = time.perf_counter()
    st = eng.save(path, build, blocking=True)
    exit_s = time.perf_counter() - t0
    fdist.barrier()
    if info.is_main:  # the box's disk holds one 48 GB file, not two
        try:
            os.remove(path)
        except OSError:
            pass
    fdist.barrier()

    # ---- loaded: steady steps, then a periodic save overlapping the following steps
    i = first_step
    evs = []

    def stamp():
        if cuda:
            ev = torch.cuda.Event(enable_timing=True)
            ev.record()
            return ev
        return time.perf_counter()

    def elapsed_ms(a, b):
        return a.elapsed_time(b) if cuda else (b - a) * 1e3

    def run(n_or_until):
        nonlocal i
        k = 0
        while True:
            step_fn(i, eng.fence)
            evs.append(stamp())
            i += 1
            k += 1
            if isinstance(n_or_until, int):
                if k >= n_or_until:
                    return k
            else:
                # one decision for every rank (each step runs collectives)
                stop = n_or_until() or k >= max_loaded_steps
                if info.world_size > 1:
                    stop = fdist.ctrl_allreduce_sum(1.0 if stop else 0.0) >= info.world_size
                if stop:
                    return k

    run(1)
    run(steady_steps)
    n_steady = len(evs)
    optimizer.gate.wait_all()  # the snapshot follows the last step's updates (as in the trainer)
    t_save = time.perf_counter()
    eng.save(path, build, blocking=False)
    enqueue_s = time.perf_counter() - t_save
    done = {}

    def finished():
        if "st" not in done:
            s = eng.poll()
            if s is not None:
                done["st"] = s
                done["k"] = 0
            return False
        done["k"] += 1
        return done["k"] >= 2  # two steady steps after the file is durable

    run(finished)
    sync()
    dts = [elapsed_ms(evs[j - 1], evs[j]) for j in range(1, len(evs))]
    steady = dts[: n_steady - 1]
    loaded = dts[n_steady - 1:]
    med = statistics.median(steady)
    visible_ms = sum(max(0.0, d - med) for d in loaded)
    ls = done.get("st")
    try:
        os.remove(path)
    except OSError:
        pass
    return {
        "bytes": st.bytes,
        "mode": eng.mode,
        "hbm_in_use_gb_at_save": round(torch.cuda.memory_reserved(dev) / 2**30, 1) if cuda else None,
        "pinned_alloc_s": round(alloc_s, 3),
        "exit_save_s": round(exit_s, 3),
        "exit_save_GB_per_s": round(st.bytes / exit_s / 1e9, 2),
        "vs_baseline_save": round(33.55 / exit_s, 2),
        "loaded": {
            "steady_step_ms": round(med, 2),
            "steps_until_durable": len(loaded),
            "step_ms_during_save_first8": [round(d, 1) for d in loaded[:8]],
            "max_step_ms_during_save": round(max(loaded), 1) if loaded else None,
            "enqueue_s": round(enqueue_s, 4),
            "save_to_durable_s": round(ls.total_s, 3) if ls is not None else None,
            "visible_s": round(visible_ms / 1e3, 4),
        },
    }
