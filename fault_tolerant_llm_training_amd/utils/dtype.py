"""Default-dtype context (reference ``utils.py:100-110``)."""
from __future__ import annotations

from contextlib import contextmanager

import torch

from .config import PRECISION_STR_TO_DTYPE  # noqa: F401  (re-export, reference utils.py:14-19)


@contextmanager
def set_default_dtype(dtype: torch.dtype):
    old = torch.get_default_dtype()
    torch.set_default_dtype(dtype)
    try:
        yield
    finally:
        torch.set_default_dtype(old)
