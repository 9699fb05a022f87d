"""Fast host→HBM restore of flat buffers from a memory-mapped checkpoint.

``torch.load(mmap=True)`` gives CPU tensors backed by the checkpoint file. A plain
``gpu.copy_(cpu)`` from pageable memory is a single-threaded staged copy, and when
the file is not in the page cache (the writer uses O_DIRECT) every 4 KiB page is a
fault served by readahead: ~2 GB/s measured on the MI355X box (48 GB of Llama-3-8B
state in ~26 s). Here a small ring of pinned chunks is filled either

* straight from the file (the tensor's file offset comes from ``/proc/self/maps``):
  the native :class:`FileReader` splits each chunk over threads issuing large
  O_DIRECT ``pread``s, or
* from memory by a pool of threads (page cache / anonymous memory → pinned memcpy;
  ATen releases the GIL),

while the previous chunks are in flight to HBM with ``hipMemcpyAsync`` on a copy
stream — disk, pinning and PCIe transfer overlap.
"""
from __future__ import annotations

import concurrent.futures as cf
import os
from typing import Dict, Optional, Tuple

import torch

CHUNK_BYTES = 256 << 20
RING = 4


class _Ring:
    def __init__(self, device: torch.device, chunk_bytes: int = CHUNK_BYTES, depth: int = RING, threads: int = 8):
        self.device = device
        self.chunk = chunk_bytes
        self.bufs = [torch.empty(chunk_bytes, dtype=torch.uint8, pin_memory=True) for _ in range(depth)]
        self.events = [None] * depth
        self.stream = torch.cuda.Stream(device=device)
        self.pool = cf.ThreadPoolExecutor(max_workers=threads)
        self.threads = threads

    def close(self):
        self.pool.shutdown(wait=True)

    def copy(self, dst: torch.Tensor, src: torch.Tensor, reader=None, file_off: int = 0) -> None:
        """dst (contiguous, on device) ← src (contiguous CPU, same dtype/numel); with a
        ``reader`` the bytes are read from its file at ``file_off`` instead of from src."""
        d = dst.reshape(-1).view(torch.uint8)
        s = src.reshape(-1).view(torch.uint8)
        n = s.numel()
        k = 0
        for off in range(0, n, self.chunk):
            ln = min(self.chunk, n - off)
            i = k % len(self.bufs)
            if self.events[i] is not None:
                self.events[i].synchronize()  # the chunk that used this buffer has landed in HBM
            buf = self.bufs[i][:ln]
            if reader is not None:
                reader.read(file_off + off, buf.data_ptr(), ln)
            else:
                part = (ln + self.threads - 1) // self.threads
                futs = [self.pool.submit(buf[a : a + part].copy_, s[off + a : off + min(ln, a + part)])
                        for a in range(0, ln, part)]
                for f in futs:
                    f.result()
            with torch.cuda.stream(self.stream):
                d[off : off + ln].copy_(buf, non_blocking=True)
                ev = torch.cuda.Event()
                ev.record(self.stream)
            self.events[i] = ev
            k += 1

    def finish(self):
        self.stream.synchronize()


_RING: Optional[_Ring] = None
_READERS: Dict[str, object] = {}
STATS = {"file_bytes": 0, "direct_bytes": 0, "memory_bytes": 0}


def file_backing(t: torch.Tensor) -> Optional[Tuple[str, int]]:
    """(path, byte offset) of the file a CPU tensor's memory maps, from ``/proc/self/maps``
    (``torch.load(mmap=True)`` maps the whole checkpoint once); None if anonymous."""
    addr = t.data_ptr()
    try:
        with open("/proc/self/maps") as f:
            for line in f:
                parts = line.split(None, 5)
                if len(parts) < 6 or not parts[5].startswith("/"):
                    continue
                lo, hi = (int(x, 16) for x in parts[0].split("-"))
                if lo <= addr < hi:
                    path = parts[5].strip()
                    if path.endswith(" (deleted)") or not os.path.isfile(path):
                        return None
                    return path, addr - lo + int(parts[2], 16)
    except OSError:
        return None
    return None


def _reader(path: str):
    r = _READERS.get(path)
    if r is None:
        from .._native import runtime, runtime_available

        if not runtime_available():
            return None
        r = runtime().FileReader(path, int(os.environ.get("FT_RESTORE_THREADS", "8")), True)
        _READERS[path] = r
    return r


def h2d(dst: torch.Tensor, src: torch.Tensor, min_bytes: int = 4 * CHUNK_BYTES) -> None:
    """Copy a (large) CPU tensor into a device tensor; plain ``copy_`` off-GPU or when small."""
    global _RING
    nbytes = src.numel() * src.element_size()
    if not dst.is_cuda or nbytes < min_bytes:
        dst.copy_(src.reshape(dst.shape) if src.shape != dst.shape else src)
        return
    if _RING is None or _RING.device != dst.device:
        _RING = _Ring(dst.device)
    reader, off = None, 0
    if src.is_contiguous() and os.environ.get("FT_RESTORE_PREAD", "1") != "0":
        fb = file_backing(src)
        if fb is not None:
            reader, off = _reader(fb[0]), fb[1]
    if reader is not None:
        d0 = reader.direct_bytes
        _RING.copy(dst, src, reader, off)
        STATS["file_bytes"] += nbytes
        STATS["direct_bytes"] += reader.direct_bytes - d0
    else:
        _RING.copy(dst, src)
        STATS["memory_bytes"] += nbytes
    _RING.finish()
    torch.cuda.current_stream(dst.device).wait_stream(_RING.stream)


def release() -> None:
    """Free the pinned ring and the file readers (after resume)."""
    global _RING
    if _RING is not None:
        _RING.finish()
        _RING.close()
        _RING = None
    _READERS.clear()
