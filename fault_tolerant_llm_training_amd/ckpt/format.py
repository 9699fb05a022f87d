"""Checkpoint file format: the reference's layout, written natively.

On-disk contract (reference ``utils.py:74-80`` / ``train.py:20-24``):

* path ``{checkpoint_path}/checkpoint_{JOBID}.ckpt``;
* one ``torch.save``-compatible zip archive holding a dict with the keys
  ``model`` (``Transformer.state_dict()`` keys), ``optimizer`` (torch AdamW
  ``state_dict`` structure), ``lr_scheduler`` (``LambdaLR.state_dict()``) and
  ``training_step`` (index of the next batch to run);
* loadable with plain ``torch.load(path, map_location="cpu")`` — including
  ``weights_only=True`` — so the reference's loader reads our files and ours
  reads theirs.

Additive keys (ignored by the reference loader): ``data_loader`` (resumable
dataset position, per rank), ``rng`` and ``meta`` (format tag, model config,
flat layout, world size).

What is different is *how* the archive is produced: the state lives in three
flat buffers (parameters, ``exp_avg``, ``exp_avg_sq``), so the archive holds
three large storages that every ``state_dict`` tensor views with an offset.
``data.pkl`` is produced here with the standard pickler (``persistent_id`` →
storage records, the same protocol ``torch.save`` uses) and the storages are
streamed from (pinned) host memory by the native multi-threaded
:class:`ZipWriter` (``csrc/runtime/zip_writer.cpp``): parallel CRC + pwrite,
fsync, atomic rename — the reference's ``torch.save`` writes non-atomically to
the final path.
"""
from __future__ import annotations

import io
import os
import pickle
import sys
from typing import Any, Dict, List, Tuple

import torch

FORMAT_TAG = "ftamd-ckpt-1"
ARCHIVE = "checkpoint"


def checkpoint_file(checkpoint_path: str, job_id) -> str:
    """``{checkpoint_path}/checkpoint_{JOBID}.ckpt`` (reference utils.py:80, train.py:22)."""
    return os.path.join(checkpoint_path, f"checkpoint_{job_id}.ckpt")


def _storage_info(obj):
    if isinstance(obj, torch.storage.TypedStorage):
        st = obj._untyped_storage
        return st, getattr(torch, obj._pickle_storage_type()), obj._size(), obj.dtype
    st = obj
    return st, torch.storage.UntypedStorage, st.nbytes(), torch.uint8


def pickle_with_storages(obj: Any) -> Tuple[bytes, List[Tuple[str, torch.UntypedStorage]]]:
    """Pickle ``obj`` like ``torch.save`` does; return (data.pkl bytes, [(key, storage)])."""
    keys: Dict[int, str] = {}
    storages: List[Tuple[str, torch.UntypedStorage]] = []
    dtypes: Dict[int, torch.dtype] = {}

    class _Pickler(pickle.Pickler):
        def persistent_id(self, o):
            if not (isinstance(o, torch.storage.TypedStorage) or torch.is_storage(o)):
                return None
            st, stype, numel, dtype = _storage_info(o)
            if st.device.type != "cpu":
                raise ValueError("checkpoint tensors must be host tensors (snapshot first)")
            ptr = st.data_ptr()
            if ptr in dtypes and dtypes[ptr] != dtype:
                raise RuntimeError("cannot save views of one storage with different dtypes")
            dtypes[ptr] = dtype
            k = keys.get(st._cdata)
            if k is None:
                k = str(len(keys))
                keys[st._cdata] = k
                storages.append((k, st))
            return ("storage", stype, k, "cpu", numel)

    buf = io.BytesIO()
    _Pickler(buf, protocol=2).dump(obj)
    return buf.getvalue(), storages


def archive_records(obj: Any) -> Tuple[List[Tuple[str, bytes]], List[Tuple[str, torch.UntypedStorage]]]:
    """Small records + storage records of a torch.save-format archive for ``obj``."""
    pkl, storages = pickle_with_storages(obj)
    small = [
        ("data.pkl", pkl),
        (".format_version", b"1"),
        (".storage_alignment", b"64"),
        ("byteorder", sys.byteorder.encode()),
    ]
    tail = [("version", b"3\n"), (".data/serialization_id", os.urandom(20).hex().encode())]
    return small + tail, storages


def write_archive_python(obj: Any, final_path: str, fsync: bool = True) -> int:
    """Pure-Python fallback (no native runtime): torch.save to a temp file, fsync, rename."""
    tmp = final_path + ".tmp"
    with open(tmp, "wb") as f:
        torch.save(obj, f)
        f.flush()
        if fsync:
            os.fsync(f.fileno())
    os.replace(tmp, final_path)
    if fsync:
        _fsync_dir(os.path.dirname(final_path) or ".")
    return os.path.getsize(final_path)


def _fsync_dir(d: str) -> None:
    try:
        fd = os.open(d, os.O_RDONLY | os.O_DIRECTORY)
    except OSError:
        return
    try:
        os.fsync(fd)
    finally:
        os.close(fd)


def strip_compile_prefix(sd: Dict[str, Any]) -> Dict[str, Any]:
    """Remove ``torch.compile``'s ``_orig_mod.`` key prefix."""
    p = "_orig_mod."
    return {(k[len(p):] if k.startswith(p) else k): v for k, v in sd.items()}


def load_checkpoint(path: str, mmap: bool = True) -> Dict[str, Any]:
    """``torch.load`` on the CPU without executing code from the file (weights_only).

    ``mmap=True`` maps the storages instead of reading 48 GB into anonymous memory,
    so restoring streams straight from the page cache into HBM.
    """
    try:
        return torch.load(path, map_location="cpu", weights_only=True, mmap=mmap)
    except RuntimeError:
        if not mmap:
            raise
        return torch.load(path, map_location="cpu", weights_only=True)
