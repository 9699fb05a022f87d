"""Tokenizer loading (reference ``train.py:28``: ``AutoTokenizer.from_pretrained``).

GPU boxes and CI have no network, so besides any Hugging Face tokenizer (hub id
or local directory) the name ``byte`` selects a dependency-free byte-level
tokenizer with the same call surface the datasets use. Tokenizing goes through
:func:`encode`, which works with both the transformers-4 ``encode_plus`` API the
reference calls (dataset.py:29-35, 80-87) and the transformers-5 ``__call__``.
"""
from __future__ import annotations

from typing import Dict, List, Optional


class ByteTokenizer:
    """UTF-8 bytes + 3 specials: pad=0, bos=1 (prepended, like Mistral's), eos=2."""

    pad_token_id = 0
    bos_token_id = 1
    eos_token_id = 2
    offset = 3
    vocab_size = 256 + 3
    name_or_path = "byte"

    def __call__(self, text: str, max_length: Optional[int] = None, padding=False, truncation: bool = False,
                 padding_side: str = "right", **_unused) -> Dict[str, List[int]]:
        ids = [self.bos_token_id] + [b + self.offset for b in text.encode("utf-8")]
        if truncation and max_length is not None:
            ids = ids[:max_length]
        if padding == "max_length" and max_length is not None and len(ids) < max_length:
            pad = [self.pad_token_id] * (max_length - len(ids))
            ids = ids + pad if padding_side == "right" else pad + ids
        return {"input_ids": ids}

    encode_plus = __call__

    def decode(self, ids) -> str:
        return bytes(i - self.offset for i in ids if i >= self.offset).decode("utf-8", errors="replace")

    def __len__(self) -> int:
        return self.vocab_size


def load_tokenizer(name_or_path: str):
    """``byte`` → :class:`ByteTokenizer`; anything else → ``AutoTokenizer.from_pretrained``."""
    if name_or_path in ("byte", "bytes"):
        return ByteTokenizer()
    from transformers import AutoTokenizer

    return AutoTokenizer.from_pretrained(name_or_path)


def encode(tokenizer, text: str, **kw) -> List[int]:
    """``input_ids`` of ``text`` (encode_plus when the tokenizer still has it, else ``__call__``)."""
    fn = getattr(tokenizer, "encode_plus", None) or tokenizer
    return list(fn(text, **kw)["input_ids"])


def pad_token_id(tokenizer) -> int:
    pid = getattr(tokenizer, "pad_token_id", None)
    if pid is None:  # many LM tokenizers have no pad token; the reference assumes one exists
        pid = getattr(tokenizer, "eos_token_id", None)
    return -1 if pid is None else int(pid)
