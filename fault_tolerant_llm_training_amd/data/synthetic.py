"""Deterministic synthetic token stream (offline GPU boxes, benchmarks, tests).

Sample ``g`` (global index) is a pure function of ``(seed, g)``, so the stream
can be resumed at any step in O(1) and sharded across data-parallel ranks
without coordination: rank ``r`` of ``W`` reads global samples
``(step * W + r) * B + j``.
"""
from __future__ import annotations

import torch


class SyntheticTokens:
    def __init__(self, vocab_size: int, seq_len: int, seed: int = 0, rank: int = 0, world_size: int = 1,
                 pin: bool = True):
        self.vocab_size = vocab_size
        self.seq_len = seq_len
        self.seed = seed
        self.rank = rank
        self.world_size = world_size
        self.pin = pin and torch.cuda.is_available()

    def sample(self, g: int) -> torch.Tensor:
        gen = torch.Generator().manual_seed(self.seed * 1_000_003 + g)
        return torch.randint(0, self.vocab_size, (self.seq_len + 1,), generator=gen)

    def batch(self, step: int, batch_size: int):
        """(inputs [B,S], labels [B,S]) for this rank at ``step`` (CLM shift like CollatorForCLM)."""
        base = (step * self.world_size + self.rank) * batch_size
        ids = torch.stack([self.sample(base + j) for j in range(batch_size)])
        inputs = ids[:, :-1].contiguous()
        labels = ids[:, 1:].contiguous()
        if self.pin:
            inputs, labels = inputs.pin_memory(), labels.pin_memory()
        return inputs, labels
