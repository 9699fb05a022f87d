"""Parquet text datasets and the causal-LM collator, with resumable state.

Behavioural parity with the reference:

* :class:`ParquetDataset` — reference ``dataset.py:10-35``: memory-mapped parquet
  table, ``len == training_samples``, item ``idx`` tokenizes row
  ``idx % num_rows`` to exactly ``S+1`` ids (right padding, truncation).
* :class:`CollatorForCLM` — reference ``dataset.py:38-53``: ``[B, S+1]`` ids →
  ``inputs = ids[:, :-1]``, ``labels = ids[:, 1:]`` with pad labels → ``-100``.
* :class:`IterableParquetDataset` — reference ``dataset.py:56-101``: packs
  successive documents into ``S+1`` tokens, re-reads the last (truncated)
  document for the next sample, masks labels at / after BOS. One fix: a
  document that alone fills a sample is not re-read (the reference would
  repeat it forever).

Additions: both datasets expose ``state_dict()`` /
``load_state_dict()`` so a resumed job seeks in O(1) instead of re-tokenizing
``training_step`` batches (reference ``train.py:36-39``), and both can be
sharded over data-parallel ranks (``rank``/``world_size``) — rank ``r`` of ``W``
reads documents ``r, r+W, r+2W, …`` (iterable) or global samples
``(step·W + r)·B + j`` (map-style, see ``data.loader``). ``world_size == 1``
reproduces the reference's single-process order exactly.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, List, Sequence

import torch

from .tokenizer import encode

IGNORE_INDEX = -100


def _read_table(path: str):
    import pyarrow.parquet as pq

    return pq.read_table(path, memory_map=True)


class _TextColumn:
    """Random access to the ``text`` column without materialising python strings up front."""

    def __init__(self, path: str):
        self.table = _read_table(path)
        self.column = self.table["text"]
        self.num_rows = len(self.table)
        if self.num_rows == 0:
            raise ValueError(f"{path}: empty parquet table")

    def __getitem__(self, i: int) -> str:
        return str(self.column[i % self.num_rows])


class ParquetDataset(torch.utils.data.Dataset):
    def __init__(self, parquet_file: str, tokenizer, sequence_length: int, training_samples: int):
        self.texts = _TextColumn(parquet_file)
        self.real_length = self.texts.num_rows
        self.tokenizer = tokenizer
        self.sequence_length = sequence_length
        self.training_samples = training_samples

    def __len__(self) -> int:
        return self.training_samples

    def __getitem__(self, idx: int) -> Dict[str, List[int]]:
        ids = encode(self.tokenizer, self.texts[idx], max_length=self.sequence_length + 1,
                     padding="max_length", truncation=True, padding_side="right")
        return {"input_ids": ids}


@dataclass
class CollatorForCLM:
    sequence_length: int
    pad_token_id: int

    def __call__(self, examples: Sequence[Dict[str, List[int]]]):
        ids = torch.tensor([e["input_ids"] for e in examples], dtype=torch.long)
        inputs = ids[:, :-1].clone()
        labels = ids[:, 1:].clone()
        labels[labels == self.pad_token_id] = IGNORE_INDEX
        assert inputs.shape[1] == labels.shape[1] == self.sequence_length
        assert inputs.shape == labels.shape
        return inputs, labels


class IterableParquetDataset(torch.utils.data.IterableDataset):
    """Packing dataset with resumable position (``current_index``)."""

    def __init__(self, parquet_file: str, tokenizer, sequence_length: int, bos_token_id: int = 1,
                 rank: int = 0, world_size: int = 1):
        self.texts = _TextColumn(parquet_file)
        self.real_length = self.texts.num_rows
        self.tokenizer = tokenizer
        self.sequence_length = sequence_length
        self.bos_token_id = bos_token_id
        self.rank = rank
        self.world_size = world_size
        self.current_index = 0  # local document counter (row = current_index*W + rank)
        self.samples = 0
        self.token_buffer: List[int] = []
        self._restored = False

    def _row(self, local_index: int) -> int:
        return (local_index * self.world_size + self.rank) % self.real_length

    def __iter__(self):
        # the reference resets its position on every iter(); a restored state survives one iter()
        if not self._restored:
            self.current_index = 0
            self.samples = 0
        self._restored = False
        self.token_buffer = []
        return self

    def __next__(self):
        S1 = self.sequence_length + 1
        buf: List[int] = []
        docs = 0
        while len(buf) < S1:
            buf.extend(encode(self.tokenizer, self.texts[self._row(self.current_index)],
                              padding=False, truncation=True, max_length=S1))
            self.current_index += 1
            docs += 1
        # the last document was cut: start the next sample from its beginning again.
        # (The reference always steps back, so a single document of ≥ S+1 tokens is
        # repeated forever; stepping back only when the sample packed more than one
        # document keeps its order otherwise and guarantees progress.)
        if docs > 1:
            self.current_index -= 1
        buf = buf[:S1]
        self.token_buffer = buf
        self.samples += 1
        t = torch.tensor(buf, dtype=torch.long)
        inputs = t[:-1].clone()
        labels = t[1:].clone()
        labels[inputs == self.bos_token_id] = IGNORE_INDEX
        labels[labels == self.bos_token_id] = IGNORE_INDEX
        return inputs, labels

    # -------------------------------------------------------------- resumable state
    def state_dict(self) -> Dict[str, int]:
        return {"current_index": int(self.current_index), "samples": int(self.samples),
                "rank": int(self.rank), "world_size": int(self.world_size)}

    def load_state_dict(self, sd: Dict[str, int]) -> None:
        if int(sd.get("world_size", self.world_size)) != self.world_size:
            raise ValueError(
                f"IterableParquetDataset state was saved with world_size={sd.get('world_size')} "
                f"but this run has world_size={self.world_size}"
            )
        self.current_index = int(sd["current_index"])
        self.samples = int(sd.get("samples", 0))
        self.token_buffer = []
        self._restored = True
