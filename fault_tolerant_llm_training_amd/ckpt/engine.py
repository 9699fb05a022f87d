"""Asynchronous checkpoint engine: HBM snapshot → pinned host → parallel file writer.

The reference saves with a synchronous ``torch.save`` of CUDA tensors (reference
``utils.py:74-80``): a pageable D2H per tensor inside pickling, then a
single-threaded write straight to the final path — ≈33.6 s for the 48 GB
Llama-3-8B state, during which training is stopped.

Here the whole training state is three flat HBM buffers (parameters,
``exp_avg``, ``exp_avg_sq``), so a checkpoint is three big DMA copies:

1. ``snapshot`` — on a dedicated HIP stream that first waits for the compute
   stream (event), copy the buffers into a reserved HBM staging area
   (``mode="hbm"``: 48 GB at HBM3E speed ≈ 20 ms; MI355X's 288 GB holds the
   64 GB of training state plus this copy), or directly into pinned host memory
   (``mode="host"``). The compute stream is made to wait for the snapshot event
   only right before the next optimizer step would overwrite the state
   (:meth:`fence`), so forward/backward of the next step overlap the copy.
2. ``drain`` — D2H of the staging copy into exact-size pinned host buffers
   (``hipHostMalloc``) on the same side stream; training never waits for it.
3. ``write`` — the native :class:`ZipWriter` thread waits for the drain event,
   then CRCs and ``pwrite``s 64 MiB chunks with a thread pool, fsyncs and
   atomically renames the file into place.

With data parallelism the save is **sharded**: every rank snapshots and writes
only its own byte ranges of the one checkpoint file (under ZeRO-1 its AdamW
shards plus 1/W of the parameters; with replicated state 1/W of everything),
straight into the file rank 0 pre-allocated, in parallel with O_DIRECT. Rank 0
pickles the state dict against zero-cost placeholder storages (a sparse-file
mapping), lays the archive out, gathers every piece's CRC32, combines them per
record (zlib ``crc32_combine``) and writes the headers/central directory, then
renames. No rank ever holds the full optimizer state and D2H/disk bandwidth
scale with W.

CPU tensors (tests, ``--device cpu``) take the same path with a synchronous
host copy. Without the native runtime the writer falls back to ``torch.save``
(temp file + fsync + rename) on a Python thread.
"""
from __future__ import annotations

import os
import tempfile
import threading
import time
from dataclasses import dataclass, field
from typing import Any, Callable, Dict, List, Optional, Tuple

import torch.distributed as dist

import torch

from .._native import runtime, runtime_available
from .format import ARCHIVE, archive_records, write_archive_python


@dataclass
class SaveStats:
    path: str = ""
    step: int = -1
    mode: str = ""
    bytes: int = 0
    snapshot_s: float = 0.0      # host time to enqueue the snapshot (+ its completion when blocking)
    stall_s: float = 0.0         # time the training loop was blocked by this save
    drain_wait_s: float = 0.0    # writer thread waiting for the D2H drain
    write_s: float = 0.0         # CRC + pwrite
    fsync_s: float = 0.0         # fsync + rename (+ dir fsync)
    direct_bytes: int = 0        # bytes written with O_DIRECT from the pinned snapshot
    total_s: float = 0.0         # save() call → file durable
    error: str = ""

    def as_dict(self) -> Dict[str, Any]:
        return dict(self.__dict__)


@dataclass
class Region:
    """This rank's part of one flat state buffer.

    ``data`` is a contiguous 1-D tensor (device or CPU) holding the rank's values;
    ``pieces`` are (flat_lo, data_off, numel): element ``data[data_off + i]`` is element
    ``flat_lo + i`` of the full buffer of ``full_numel`` elements.
    """

    name: str
    data: torch.Tensor
    pieces: List[Tuple[int, int, int]]
    full_numel: int

    @staticmethod
    def whole(name: str, t: torch.Tensor) -> "Region":
        return Region(name, t, [(0, 0, t.numel())], t.numel())

    @property
    def is_whole(self) -> bool:
        return self.pieces == [(0, 0, self.full_numel)] and self.data.numel() == self.full_numel


def placeholder(numel: int, dtype: torch.dtype) -> torch.Tensor:
    """A CPU tensor of ``numel`` elements backed by a sparse-file private mapping: valid for
    pickling (size, dtype, identity) yet using no memory, since its pages are never touched."""
    nbytes = numel * torch.empty((), dtype=dtype).element_size()
    fd, path = tempfile.mkstemp(prefix="ftckpt_ph_")
    try:
        os.ftruncate(fd, max(nbytes, 1))
        os.close(fd)
        st = torch.UntypedStorage.from_file(path, False, max(nbytes, 1))
    finally:
        os.unlink(path)
    return torch.empty(0, dtype=dtype).set_(st)[:numel]


@dataclass
class _InFlight:
    stats: SaveStats
    t0: float
    writer: Any = None                    # native ZipWriter
    thread: Optional[threading.Thread] = None  # python fallback writer
    keep: List[Any] = field(default_factory=list)  # host tensors referenced by the writer
    done: bool = False


class CheckpointEngine:
    def __init__(self, buffers, mode: str = "auto", writer_threads: int = 8,
                 fsync: bool = True, hbm_headroom_gb: float = 16.0, group=None, rank: int = 0, world: int = 1,
                 sharded: Optional[bool] = None):
        """``buffers``: name → flat device (or CPU) tensor holding training state (single
        writer), or a list of :class:`Region` (this rank's pieces; ``world`` > 1 → sharded
        save over the gloo ``group``)."""
        if isinstance(buffers, dict):
            self.regions = [Region.whole(k, v) for k, v in buffers.items()]
        else:
            self.regions = list(buffers)
        self.rank, self.world, self.group = rank, world, group
        self.sharded = world > 1 if sharded is None else sharded
        if not self.sharded and not all(r.is_whole for r in self.regions):
            raise ValueError("a single-writer engine needs whole buffers")
        self.buffers = {r.name: r.data for r in self.regions}
        self.device = next(iter(self.buffers.values())).device
        self.is_cuda = self.device.type == "cuda"
        self.native = runtime_available()
        self.writer_threads = writer_threads
        self.fsync = fsync
        self.nbytes = sum(b.numel() * b.element_size() for b in self.buffers.values())  # this rank's share
        self.full_nbytes = sum(r.full_numel * r.data.element_size() for r in self.regions)
        # "auto" is resolved at first use (the first save, or an explicit preallocate()), not
        # here: an engine built at startup to pin its host buffers early must not reserve an
        # HBM staging copy that the activations of a long-context run need
        self._mode = "cpu" if not self.is_cuda else mode
        self._hbm_headroom = hbm_headroom_gb
        self._host: Optional[Dict[str, torch.Tensor]] = None
        self._stage: Optional[Dict[str, torch.Tensor]] = None
        self._eng = None
        self._snap_ev: Optional[int] = None
        self._inflight: Optional[_InFlight] = None
        self.history: List[SaveStats] = []
        self._host_lock = threading.Lock()
        self._prealloc: Optional[threading.Thread] = None
        self.prealloc_s: Optional[float] = None

    @property
    def mode(self) -> str:
        if self._mode == "auto":
            free, _total = torch.cuda.mem_get_info(self.device)
            self._mode = "hbm" if free > self.nbytes + self._hbm_headroom * 2**30 else "host"
        return self._mode

    # ------------------------------------------------------------------ buffers
    def _ensure_host(self) -> Dict[str, torch.Tensor]:
        with self._host_lock:  # a save waits here for a background preallocation in flight
            return self._ensure_host_locked()

    def _ensure_host_locked(self) -> Dict[str, torch.Tensor]:
        if self._host is None:
            host = {}
            for k, b in self.buffers.items():
                nb = b.numel() * b.element_size()
                if self.is_cuda and self.native:
                    # exact size (torch's pinned pool rounds to 2^k), pinned for this rank's GPU
                    raw = runtime().pinned_empty(nb, self.device.index or 0)
                elif self.is_cuda:
                    raw = torch.empty(nb, dtype=torch.uint8, pin_memory=True)
                else:
                    raw = torch.empty(nb, dtype=torch.uint8)
                host[k] = raw.view(b.dtype)
            self._host = host
        return self._host

    def _ensure_stage(self) -> Dict[str, torch.Tensor]:
        if self._stage is None:
            self._stage = {k: torch.empty_like(b) for k, b in self.buffers.items()}
        return self._stage

    def preallocate(self) -> None:
        """Allocate pinned host (and HBM staging) buffers ahead of the first save."""
        self._ensure_host()
        if self.mode == "hbm":
            self._ensure_stage()

    def preallocate_async(self) -> None:
        """Same, with the pinned host buffers allocated by a background thread while training
        runs: pinning 48 GB takes ~3.3 s on the MI355X box, which would otherwise sit inside the
        first save — the SIGUSR1 one, against the Slurm deadline (reference train.sh:12). The
        HBM staging copy (``hbm`` mode) stays lazy: it is a fast device allocation, and "auto"
        decides on it at the first save. A save that starts before the thread is done blocks on
        the host-buffer lock."""
        if self._host is not None or self._prealloc is not None:
            return

        def run():
            t0 = time.perf_counter()
            if self.is_cuda:
                torch.cuda.set_device(self.device)  # per-thread current device (pinned-page placement)
            self._ensure_host()
            self.prealloc_s = time.perf_counter() - t0

        self._prealloc = threading.Thread(target=run, name="ckpt-prealloc", daemon=True)
        self._prealloc.start()

    def preallocated(self, timeout: Optional[float] = None) -> bool:
        """Wait up to ``timeout`` s for a background preallocation; True once buffers exist."""
        if self._prealloc is not None:
            self._prealloc.join(timeout)
        return self._host is not None

    def host_views(self) -> Dict[str, torch.Tensor]:
        return self._ensure_host()

    # ------------------------------------------------------------------ snapshot
    def _snapshot(self) -> Optional[int]:
        """Enqueue the copies; returns the native event index the writer must wait on."""
        host = self._ensure_host()
        if not self.is_cuda:
            for k, b in self.buffers.items():
                host[k].copy_(b)
            return None
        if not self.native:
            # no native engine: synchronous pinned copies on the current stream
            for k, b in self.buffers.items():
                host[k].copy_(b, non_blocking=True)
            torch.cuda.current_stream(self.device).synchronize()
            return None
        rt = runtime()
        if self._eng is None:
            self._eng = rt.SnapshotEngine(self.device.index or 0)
        eng = self._eng
        eng.begin(torch.cuda.current_stream(self.device).cuda_stream)
        if self.mode == "hbm":
            stage = self._ensure_stage()
            for k, b in self.buffers.items():
                eng.copy(stage[k].data_ptr(), b.data_ptr(), b.numel() * b.element_size())
            self._snap_ev = eng.mark()
            src = stage
        else:
            src = self.buffers
        for k, b in src.items():
            eng.copy(host[k].data_ptr(), b.data_ptr(), b.numel() * b.element_size())
        drained = eng.mark()
        if self.mode != "hbm":
            self._snap_ev = drained
        return drained

    def fence(self) -> None:
        """Make the compute stream wait for the pending snapshot (call before optimizer.step)."""
        if self._snap_ev is not None and self._eng is not None:
            if not self._eng.query(self._snap_ev):
                self._eng.stream_wait(torch.cuda.current_stream(self.device).cuda_stream, self._snap_ev)
            self._snap_ev = None

    # ------------------------------------------------------------------ save
    def save(self, path: str, build_state: Callable[[Dict[str, torch.Tensor]], Any], step: int = -1,
             blocking: bool = False) -> SaveStats:
        """Snapshot the buffers and write ``build_state(host_views)`` to ``path``.

        ``build_state`` receives the host buffers (same keys as ``buffers``) and
        returns the object to serialise; its tensors must be views of them (or
        small CPU tensors). Returns immediately unless ``blocking``.
        """
        t0 = time.perf_counter()
        self.wait()  # host buffers are reused: the previous file must be on disk
        st = SaveStats(path=path, step=step, mode=self.mode, bytes=self.full_nbytes)
        os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
        ev = self._snapshot()
        inf = _InFlight(stats=st, t0=t0)
        tmp = path + ".tmp"
        if self.sharded:
            self._save_sharded(path, tmp, build_state, ev, inf)
        elif self.native:
            obj = build_state(self._ensure_host())
            rt = runtime()
            small, storages = archive_records(obj)
            w = rt.ZipWriter(tmp, path, ARCHIVE, self.writer_threads)
            for name, data in small[:4]:
                w.add_bytes(name, data)
            for key, storage in storages:
                w.add_buffer(f"data/{key}", storage.data_ptr(), storage.nbytes())
                inf.keep.append(storage)
            for name, data in small[4:]:
                w.add_bytes(name, data)
            handle = self._eng.event_handle(ev) if (ev is not None and self._eng is not None) else 0
            w.start(handle, self.fsync)
            inf.writer = w
            st.bytes = w.total_size()
        else:
            obj = build_state(self._ensure_host())

            def _py_write():
                try:
                    st.bytes = write_archive_python(obj, path, self.fsync)
                except Exception as e:  # pragma: no cover - reported through stats
                    st.error = repr(e)

            inf.thread = threading.Thread(target=_py_write, name="ft-ckpt-writer", daemon=True)
            inf.thread.start()
            inf.keep.append(obj)
        st.snapshot_s = time.perf_counter() - t0
        self._inflight = inf
        if blocking:
            if self.is_cuda and self._snap_ev is not None:
                self.fence()
            self.wait()
        st.stall_s = time.perf_counter() - t0 if blocking else st.snapshot_s
        return st

    # ------------------------------------------------------------------ sharded save
    def _save_sharded(self, path: str, tmp: str, build_state, ev, inf: _InFlight) -> None:
        if not self.native:
            raise RuntimeError("sharded checkpoint writes need the native runtime (_runtime.so)")
        rt = runtime()
        host = self._ensure_host()
        zw = None
        offs = None
        if self.rank == 0:
            ph = {r.name: placeholder(r.full_numel, r.data.dtype) for r in self.regions}
            by_ptr = {t.untyped_storage().data_ptr(): name for name, t in ph.items()}
            obj = build_state(ph)
            small, storages = archive_records(obj)
            zw = rt.ZipWriter(tmp, path, ARCHIVE, self.writer_threads)
            ext = {}
            for name, data in small[:4]:
                zw.add_bytes(name, data)
            for key, storage in storages:
                region = by_ptr.get(storage.data_ptr())
                if region is not None:
                    zw.add_external(f"data/{key}", storage.nbytes(), 0)
                    ext[f"data/{key}"] = region
                else:
                    zw.add_buffer(f"data/{key}", storage.data_ptr(), storage.nbytes())
                    inf.keep.append(storage)
            for name, data in small[4:]:
                zw.add_bytes(name, data)
            offs = {ext[name]: (name, off) for name, off, _size in zw.layout_records() if name in ext}
            if set(offs) != {r.name for r in self.regions}:
                raise RuntimeError(f"sharded save: state dict does not view every region ({sorted(offs)})")
            zw.create_file()
            inf.keep.extend(ph.values())
            st_bytes = zw.total_size()
            inf.stats.bytes = st_bytes
        handle = self._eng.event_handle(ev) if (ev is not None and self._eng is not None) else 0
        regions = self.regions
        group = self.group
        rank = self.rank
        nthreads = self.writer_threads
        fsync = self.fsync
        stats = inf.stats

        def _run():
            err = ""
            try:
                box = [offs]
                dist.broadcast_object_list(box, src=0, group=group)
                roffs = box[0]
                file_offs, ptrs, lens, meta = [], [], [], []
                for r in regions:
                    rec, base = roffs[r.name]
                    h = host[r.name]
                    es = h.element_size()
                    for flat_lo, data_off, n in r.pieces:
                        file_offs.append(base + flat_lo * es)
                        ptrs.append(h.data_ptr() + data_off * es)
                        lens.append(n * es)
                        meta.append((rec, flat_lo * es, n * es))
                t_w = time.perf_counter()
                crcs = rt.write_pieces(tmp, file_offs, ptrs, lens, nthreads, handle, fsync, True)
                stats.write_s = time.perf_counter() - t_w
                mine = [(rec, lo, ln, c) for (rec, lo, ln), c in zip(meta, crcs)]
            except Exception as e:  # report to rank 0, keep the collectives in step
                err = f"rank {rank}: {e!r}"
                mine = []
            gathered = [None] * dist.get_world_size(group) if rank == 0 else None
            dist.gather_object((err, mine), gathered, dst=0, group=group)
            status = ""
            if rank == 0:
                errs = [g[0] for g in gathered if g[0]]
                try:
                    if errs:
                        raise RuntimeError("; ".join(errs))
                    per = {}
                    for _e, pieces in gathered:
                        for rec, lo, ln, c in pieces:
                            per.setdefault(rec, []).append((lo, ln, c))
                    for rec, sizes in ((n, s_) for n, _o, s_ in zw.layout_records() if n in per):
                        ps = sorted(per[rec])
                        pos, crc = 0, None
                        for lo, ln, c in ps:
                            if lo != pos:
                                raise RuntimeError(f"{rec}: pieces do not tile the record (gap at byte {pos})")
                            crc = c if crc is None else rt.crc32_combine(crc, c, ln)
                            pos += ln
                        if pos != sizes:
                            raise RuntimeError(f"{rec}: pieces cover {pos} of {sizes} bytes")
                        zw.set_external_crc(rec, crc)
                    t_f = time.perf_counter()
                    zw.run_sync(0, fsync)
                    ws = zw.wait()
                    if ws.error:
                        raise RuntimeError(ws.error)
                    stats.fsync_s = time.perf_counter() - t_f
                except Exception as e:
                    status = repr(e)
            box = [status]
            dist.broadcast_object_list(box, src=0, group=group)
            if box[0]:
                stats.error = box[0]

        inf.thread = threading.Thread(target=_run, name="ft-ckpt-sharded", daemon=True)
        inf.thread.start()

    def poll(self) -> Optional[SaveStats]:
        """Non-blocking: if the in-flight save finished, retire it and return its stats."""
        inf = self._inflight
        if inf is None:
            return None
        if inf.writer is not None and not inf.writer.done():
            return None
        if inf.thread is not None and inf.thread.is_alive():
            return None
        return self.wait()

    def wait(self) -> Optional[SaveStats]:
        """Block until the in-flight save (if any) is durable; returns its stats."""
        inf = self._inflight
        if inf is None:
            return None
        st = inf.stats
        if inf.writer is not None:
            ws = inf.writer.wait()
            st.drain_wait_s, st.write_s, st.fsync_s = ws.wait_seconds, ws.write_seconds, ws.fsync_seconds
            st.bytes = ws.bytes or st.bytes
            st.direct_bytes = ws.direct_bytes
            if ws.error:
                st.error = ws.error
        if inf.thread is not None:
            inf.thread.join()
        st.total_s = time.perf_counter() - inf.t0
        self._inflight = None
        self.history.append(st)
        if st.error:
            raise RuntimeError(f"checkpoint write to {st.path} failed: {st.error}")
        return st

    @property
    def busy(self) -> bool:
        return self._inflight is not None
