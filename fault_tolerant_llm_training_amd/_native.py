"""Loaders for the in-tree native libraries.

GPU code paths call :func:`kernels` and fail loudly when ``_kernels.so`` is
missing — there is no silent eager fallback on the GPU. CPU tensors take the
pure-PyTorch reference implementation in each op module (that is the CPU
backend used by the gloo/CPU tests, not a GPU fallback).
"""
from __future__ import annotations

import importlib.util
import os
import threading
from pathlib import Path

import torch

_PKG = Path(__file__).resolve().parent
# FT_KERNELS_SO: load another build of the kernel library (A/B of two kernel builds in
# separate processes, scripts/flash_bench.py); unset = the in-tree build
KERNELS_SO = Path(os.environ.get("FT_KERNELS_SO") or (_PKG / "_kernels.so"))
RUNTIME_SO = _PKG / "_runtime.so"

_lock = threading.Lock()
_kernels_loaded = False
_runtime_mod = None


class NativeExtensionMissing(RuntimeError):
    pass


def _missing(path: Path) -> NativeExtensionMissing:
    return NativeExtensionMissing(
        f"native library {path.name} not found at {path}; build it with "
        "`python -m fault_tolerant_llm_training_amd._build` (hipcc --offload-arch=gfx950)"
    )


# dtypes the gfx950 kernels cover; a CUDA tensor of another dtype (fp64 models, --model-dtype fp64)
# takes the composed-PyTorch path that CPU tensors take
NATIVE_DTYPES = (torch.bfloat16, torch.float16, torch.float32)


def native(t: torch.Tensor) -> bool:
    """True when ``t`` is handled by the HIP kernels (a GPU tensor of a kernel dtype)."""
    return t.is_cuda and t.dtype in NATIVE_DTYPES


def kernels():
    """Return ``torch.ops.ftamd`` after loading ``_kernels.so`` (raises if absent)."""
    global _kernels_loaded
    if not _kernels_loaded:
        with _lock:
            if not _kernels_loaded:
                if not KERNELS_SO.exists():
                    raise _missing(KERNELS_SO)
                torch.ops.load_library(str(KERNELS_SO))
                _kernels_loaded = True
    return torch.ops.ftamd


def runtime():
    """Return the ``_runtime`` pybind11 module (signals, snapshot engine, zip writer)."""
    global _runtime_mod
    if _runtime_mod is None:
        with _lock:
            if _runtime_mod is None:
                if not RUNTIME_SO.exists():
                    raise _missing(RUNTIME_SO)
                spec = importlib.util.spec_from_file_location(
                    "fault_tolerant_llm_training_amd._runtime", str(RUNTIME_SO)
                )
                mod = importlib.util.module_from_spec(spec)
                spec.loader.exec_module(mod)
                _runtime_mod = mod
    return _runtime_mod


def runtime_available() -> bool:
    try:
        runtime()
        return True
    except Exception:
        return False
