"""Per-shape GEMM solution table for the training step's hipBLASLt/rocBLAS GEMMs.

Every projection of the step is a plain ``torch.mm``/``torch.addmm`` (ops/functional.py).
PyTorch-ROCm's TunableOp can route those calls to a specific hipBLASLt (or rocBLAS)
solution index per (layout, M, N, K, ld) instead of the library heuristic's first pick.
``scripts/tune_gemms.py`` benchmarks every candidate solution for every GEMM one
Llama-3-8B step issues on an MI355X and writes the winners to ``tuning/gemm_gfx950.csv``
(committed, like a kernel tuning table); :func:`use_tuned_gemms` loads that table with
tuning disabled, so a run never benchmarks anything (and never rewrites the table) and
shapes not in the table keep the default heuristic. TunableOp itself rejects the table
if the PyTorch / ROCm / hipBLASLt / rocBLAS versions or the GPU arch differ from the
ones it was tuned on.

``FT_TUNED_GEMM=0`` disables it (A/B); ``FT_TUNED_GEMM=<path>`` loads another table.
"""
from __future__ import annotations

import os
from typing import Optional

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
DEFAULT_DB = os.path.join(ROOT, "tuning", "gemm_gfx950.csv")

_loaded: Optional[bool] = None


def use_tuned_gemms(path: Optional[str] = None) -> bool:
    """Load the GEMM solution table (once per process). Returns True if it is active."""
    global _loaded
    if _loaded is not None:
        return _loaded
    env = os.environ.get("FT_TUNED_GEMM", "1")
    _loaded = False
    if env == "0" or not torch.cuda.is_available() or torch.version.hip is None:
        return False
    path = path or (env if env not in ("", "1") else DEFAULT_DB)
    if not os.path.exists(path):
        return False
    import torch.cuda.tunable as tunable

    tunable.tuning_enable(False)
    tunable.record_untuned_enable(False)
    tunable.enable(True)
    _loaded = bool(tunable.read_file(path))
    if not _loaded:
        tunable.enable(False)
    return _loaded


def set_enabled(on: bool) -> None:
    """Switch between the tuned table and the library heuristic (same-process A/B)."""
    import torch.cuda.tunable as tunable

    tunable.enable(on)
