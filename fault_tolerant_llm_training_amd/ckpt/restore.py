"""Fast host→HBM restore of flat buffers from a memory-mapped checkpoint.

``torch.load(mmap=True)`` gives CPU tensors backed by the page cache. A plain
``gpu.copy_(cpu)`` from pageable memory is a single-threaded staged copy
(~7 GB/s measured on the MI355X box: 48 GB of Llama-3-8B state took ~9 s). Here a
small ring of pinned chunks is filled by a pool of threads (page cache → pinned
memcpy runs in parallel; ATen releases the GIL) while the previous chunks are in
flight to HBM with ``hipMemcpyAsync`` on a copy stream — reading, pinning and PCIe
transfer overlap.
"""
from __future__ import annotations

import concurrent.futures as cf
from typing import Optional

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

    def copy(self, dst: torch.Tensor, src: torch.Tensor) -> None:
        """dst (contiguous, on device) ← src (contiguous CPU, same dtype/numel)."""
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


def h2d(dst: torch.Tensor, src: torch.Tensor, min_bytes: int = 4 * CHUNK_BYTES) -> None:
    """Copy a (large) CPU tensor into a device tensor; plain ``copy_`` off-GPU or when small."""
    global _RING
    if not dst.is_cuda or src.numel() * src.element_size() < min_bytes:
        dst.copy_(src.reshape(dst.shape) if src.shape != dst.shape else src)
        return
    if _RING is None or _RING.device != dst.device:
        _RING = _Ring(dst.device)
    _RING.copy(dst, src)
    _RING.finish()
    torch.cuda.current_stream(dst.device).wait_stream(_RING.stream)


def release() -> None:
    """Free the pinned ring (after resume)."""
    global _RING
    if _RING is not None:
        _RING.finish()
        _RING.close()
        _RING = None
