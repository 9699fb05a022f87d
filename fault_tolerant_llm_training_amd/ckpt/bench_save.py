"""Checkpoint-save timing for ``bench.py --ckpt-dir`` (BASELINE metric: save wall-clock).

Measures one save of the full training state (params + AdamW moments, the
reference's ≈48.3 GB for Llama-3-8B) through the asynchronous engine:

* ``stall_s`` — how long the training loop is blocked (snapshot enqueue, plus
  the wait for the HBM snapshot before the next optimizer step);
* ``total_s`` — save() call → file durable on disk (fsync + atomic rename),
  comparable to the reference's synchronous ``torch.save`` (33.6 s).
"""
from __future__ import annotations

import os
import time

import torch

from .engine import CheckpointEngine
from .format import checkpoint_file
from .state import build_checkpoint


def time_checkpoint_save(model, optimizer, lr_scheduler, ckpt_dir: str, info, mode: str = "auto",
                         keep: bool = False):
    if not info.is_main:
        return None
    eng = CheckpointEngine({"params": model.flat.params, "exp_avg": optimizer.exp_avg,
                            "exp_avg_sq": optimizer.exp_avg_sq}, mode=mode)
    t_alloc = time.perf_counter()
    eng.preallocate()
    alloc_s = time.perf_counter() - t_alloc
    path = checkpoint_file(ckpt_dir, "bench")
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    st = eng.save(path, lambda host: build_checkpoint(model, optimizer, lr_scheduler, 0, host), blocking=False)
    enq = time.perf_counter() - t0
    eng.fence()  # what the next optimizer step would wait for
    torch.cuda.current_stream().synchronize()  # (not the side stream's D2H drain)
    stall = time.perf_counter() - t0
    st = eng.wait()
    total = time.perf_counter() - t0
    out = {
        "mode": eng.mode,
        "bytes": st.bytes,
        "stall_s": round(stall, 4),
        "enqueue_s": round(enq, 4),
        "drain_wait_s": round(st.drain_wait_s, 3),
        "write_s": round(st.write_s, 3),
        "fsync_s": round(st.fsync_s, 3),
        "direct_GB": round(st.direct_bytes / 1e9, 2),
        "total_s": round(total, 3),
        "GB_per_s": round(st.bytes / total / 1e9, 2),
        "pinned_alloc_s": round(alloc_s, 3),
        "vs_baseline_save_s": round(33.55 / total, 2),
    }
    if not keep:
        try:
            os.remove(path)
        except OSError:
            pass
    return out
