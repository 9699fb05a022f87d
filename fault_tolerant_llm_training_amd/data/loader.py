"""Prefetching, resumable, data-parallel batch loader.

Replaces the reference's ``DataLoader(train_ds, batch_size, collate_fn)`` with
``num_workers=0`` (train.py:30-34) plus its O(steps) replay-skip on resume
(train.py:36-39):

* a producer thread tokenizes/collates the next ``prefetch`` batches into
  pinned host memory while the GPU runs the current step, so the hot loop only
  issues a non-blocking H2D copy;
* every batch carries the loader state *after* that batch, so the trainer can
  checkpoint exactly the position of the last batch it consumed (prefetched but
  unconsumed batches are simply re-produced after a resume);
* the number of loss tokens of the local batch (reference train.py:94) is
  counted on the host here; the trainer makes it global for DP (SURVEY.md
  §A.12) with a 4-byte device all-reduce that never blocks the host.

Sources: ``synthetic`` (SyntheticTokens), ``parquet`` (map-style
ParquetDataset + CollatorForCLM, O(1) seek by sample index) and ``iterable``
(IterableParquetDataset, state = document cursor).
"""
from __future__ import annotations

import queue
import threading
from dataclasses import dataclass
from typing import Any, Dict, Optional

import torch

from .parquet import IGNORE_INDEX, CollatorForCLM, IterableParquetDataset, ParquetDataset
from .synthetic import SyntheticTokens


@dataclass
class Batch:
    step: int                 # global step index this batch belongs to
    inputs: torch.Tensor      # [B, S] int64 (pinned when CUDA is available)
    labels: torch.Tensor      # [B, S] int64
    num_items: int            # loss tokens in this rank's batch
    state: Dict[str, Any]     # loader state after this batch


class _Source:
    kind = "base"

    def produce(self, step: int):
        raise NotImplementedError

    def state_after(self, step: int) -> Dict[str, Any]:
        return {"kind": self.kind, "next_step": step + 1}

    def state_before(self, step: int) -> Dict[str, Any]:
        return {"kind": self.kind, "next_step": step}

    def load_state(self, state: Dict[str, Any]) -> int:
        if state.get("kind") != self.kind:
            raise ValueError(f"data loader state is for {state.get('kind')!r}, this run uses {self.kind!r}")
        return int(state["next_step"])


class SyntheticSource(_Source):
    kind = "synthetic"

    def __init__(self, ds: SyntheticTokens, batch_size: int):
        self.ds, self.B = ds, batch_size

    def produce(self, step):
        return self.ds.batch(step, self.B)


class MapSource(_Source):
    """Global sample ``(step·W + rank)·B + j`` — for W=1 the reference DataLoader order."""

    kind = "parquet"

    def __init__(self, ds: ParquetDataset, collator: CollatorForCLM, batch_size: int, rank: int, world: int):
        self.ds, self.collator, self.B, self.rank, self.world = ds, collator, batch_size, rank, world

    def produce(self, step):
        base = (step * self.world + self.rank) * self.B
        return self.collator([self.ds[base + j] for j in range(self.B)])


class IterableSource(_Source):
    kind = "iterable"

    def __init__(self, ds: IterableParquetDataset, batch_size: int):
        self.ds, self.B = ds, batch_size
        self.it = iter(ds)
        self._states: Dict[int, Dict[str, Any]] = {}

    def produce(self, step):
        xs, ys = zip(*(next(self.it) for _ in range(self.B)))
        self._states[step] = self.ds.state_dict()
        return torch.stack(xs), torch.stack(ys)

    def state_after(self, step):
        return {"kind": self.kind, "next_step": step + 1, "dataset": self._states.pop(step)}

    def state_before(self, step):
        return {"kind": self.kind, "next_step": step, "dataset": self.ds.state_dict()}

    def load_state(self, state):
        nxt = super().load_state(state)
        self.ds.load_state_dict(state["dataset"])
        self.it = iter(self.ds)
        return nxt


class TrainLoader:
    """Iterates :class:`Batch` for steps ``start_step, start_step+1, …`` (background prefetch)."""

    def __init__(self, source: _Source, start_step: int = 0, state: Optional[Dict[str, Any]] = None,
                 prefetch: int = 2, pin: Optional[bool] = None):
        self.source = source
        self.step = source.load_state(state) if state is not None else start_step
        self.prefetch = max(0, prefetch)
        self.pin = torch.cuda.is_available() if pin is None else pin
        self._q: "queue.Queue" = queue.Queue(maxsize=max(1, self.prefetch))
        self._stop = threading.Event()
        self._thread: Optional[threading.Thread] = None
        self._next_produce = self.step
        self._initial_state = source.state_before(self.step)
        self.last_state: Optional[Dict[str, Any]] = None

    # ------------------------------------------------------------------ producer
    def _make(self, step: int) -> Batch:
        inputs, labels = self.source.produce(step)
        n = int((labels != IGNORE_INDEX).sum())
        if self.pin and not inputs.is_pinned():
            inputs, labels = inputs.pin_memory(), labels.pin_memory()
        return Batch(step, inputs, labels, n, self.source.state_after(step))

    def _run(self):
        try:
            while not self._stop.is_set():
                b = self._make(self._next_produce)
                self._next_produce += 1
                while not self._stop.is_set():
                    try:
                        self._q.put(b, timeout=0.1)
                        break
                    except queue.Full:
                        continue
        except BaseException as e:  # surface producer errors in the consumer
            self._q.put(e)

    def __iter__(self):
        return self

    def __next__(self) -> Batch:
        if self.prefetch == 0:
            b = self._make(self._next_produce)
            self._next_produce += 1
        else:
            if self._thread is None:
                self._thread = threading.Thread(target=self._run, name="ft-data-prefetch", daemon=True)
                self._thread.start()
            b = self._q.get()
            if isinstance(b, BaseException):
                raise b
        self.step = b.step + 1
        self.last_state = b.state
        return b

    def state_dict(self) -> Dict[str, Any]:
        """State after the last *consumed* batch (what a checkpoint must record)."""
        return dict(self.last_state if self.last_state is not None else self._initial_state)

    def close(self):
        self._stop.set()
        if self._thread is not None:
            self._thread.join(timeout=5)
            self._thread = None
