"""Gradient pipeline: buckets, collectives over RCCL/xGMI, overlapped grad-norm.

Every weight gradient is written straight into the flat gradient buffer by its
backward kernel/GEMM, which then calls :meth:`GradSink.ready`. Buckets are
contiguous ranges of that buffer cut at parameter boundaries in *reverse*
layout order (the order backward produces them: LM head first, embedding
last). The moment the last gradient of a bucket has been enqueued, the bucket's
work is launched while the compute stream keeps running backward:

``local``     (1 rank)  side stream: partial sum of squares of the bucket.
``allreduce`` (DP)      RCCL ``all_reduce(SUM)`` of the bucket, then its
                        partial sum of squares on the side stream.
``zero1``     (DP)      RCCL ``reduce_scatter`` of the bucket into this rank's
                        1/W shard (ZeRO-1: optimizer state is sharded), then the
                        shard's partial sum of squares. After AdamW updates the
                        shard, an ``all_gather`` republishes the bucket's
                        parameters (``optim.adamw``).

Buckets launch strictly in index order (a bucket that completes early waits for
the ones above it), so every rank issues the same collective sequence; that is
what lets a rank whose step failed half-way (:meth:`GradReducer.poison_and_complete`)
issue exactly the collectives its peers are waiting for.

Gradient accumulation (``--grad-accum K``): micro-batches ``0..K-2`` only
accumulate into the flat buffer (sinks in accumulate mode, no collectives,
embedding rows stashed); the buckets launch during the last micro-batch's
backward, so the collective volume per optimizer step is independent of K.

So the gradient norm needed for clipping (reference utils.py:58-63) is
finished a few µs after backward ends, and the optimizer (which the
reference runs as a separate serial phase, train.py:107-109) starts at once.

The token-embedding gradient is the exception: it has at most B·S nonzero rows
per rank, so instead of a dense 1 GB collective at the very end of backward
(on the critical path into the next forward), the embedding backward
all-gathers every rank's (token, dY row) pairs — 16 MB per rank for Llama-3-8B
— and scatter-adds them locally in a fixed order (sparse exchange).

The loss is normalised by the *global* token count (trainer), so SUM (not
AVG) reproduces the single-process gradient of the global batch.

Bucket size: on an 8× MI355X node every GPU has 7 xGMI links (~153 GB/s
each, point to point). A ring collective is per-link bound and RCCL only
spreads a collective over several channels/links when the message is large,
so buckets are large (default 256 MiB): Llama-3-8B's 16 GB of bf16 gradients
become ~64 collectives per step — few launches, still ~2 overlap points per
transformer layer. ZeRO-1 moves the same bytes as all-reduce (reduce-scatter +
all-gather) but each rank updates and stores only 1/W of the AdamW state: the
bandwidth-bound optimizer pass (≈20 ms for 8B params on one GPU) shrinks W×,
and 288 GB of HBM is not the limit for the replicated parameters anyway.
"""
from __future__ import annotations

import os
from typing import List, Optional

import torch
import torch.distributed as dist

from .._native import kernels, native
from ..models.flat import FlatParamSpace
from ..ops.grad_sink import GradSink

MODES = ("local", "allreduce", "zero1")
LOCAL_BUCKET_MB = 64.0
DP_BUCKET_MB = 256.0
PARTIALS_PER_BUCKET = 512
# A/B switch (scripts/ab_step.py): take every bucket's sum of squares in one pass after
# backward instead of as each bucket completes (the default overlaps them with backward)
SUMSQ_AT_END = False


def set_sumsq_at_end(on: bool) -> None:
    global SUMSQ_AT_END
    SUMSQ_AT_END = bool(on)


# One GPU ("local" mode): the gradient norm's partial sums of squares come from the kernels that
# write the gradients (the w4 dW GEMM's epilogue per output tile, the norm backward's column sums
# per 32 columns) into a per-sink slice of ``partials``; only gradients whose producer has no such
# epilogue (the embedding's scatter-add, hipBLASLt fallbacks) get the separate sumsq pass. The
# 16 GB re-read of the Llama-3-8B gradient per step is gone. set_fused_sumsq(False): per-bucket passes.
# (Under DP the norm is of the REDUCED gradient, so the passes run after each bucket's collective.)
FUSED_SUMSQ = True


def set_fused_sumsq(on: bool) -> None:
    global FUSED_SUMSQ
    FUSED_SUMSQ = bool(on)


def sink_partials(numel: int, ndim: int, shape=None, tile_rows: int = 256) -> int:
    """Partial slots a sink's producers may write: one per output tile of a 2-D weight (w4: 256 x
    >= 128, a tail tile of the dW layout covering fewer: ceil(rows / 256) x ceil(cols / 128); the
    fp32 MFMA GEMM's 128 x 128 tiles: tile_rows = 128), one per 32 columns of a 1-D one; also the grid
    of the fallback sumsq pass. (Every slot enters norm_finish's sum: no more than the producers use.)"""
    if ndim <= 1:
        return max(1, (numel + 31) // 32)
    n = max(1, (numel + 32767) // 32768)
    if shape is not None and len(shape) == 2:
        n = max(n, -(-int(shape[0]) // tile_rows) * -(-int(shape[1]) // 128))
    return n


def _copy_back(dst: torch.Tensor, src: torch.Tensor, temps) -> None:
    """fp32 reduce: round the reduced fp32 copy back into the gradient buffer.

    Runs on the stream that waited for the collective (the reducer's side stream), while the
    fp32 temporaries were allocated on the stream that launched the bucket (compute or dW
    stream). Their last Python references are dropped right after this enqueue, so they are
    recorded on the current stream: the caching allocator then keeps their blocks until this
    copy has read them, instead of handing them to the next bucket's ``grads.float()``."""
    dst.copy_(src)
    if src.is_cuda:
        cur = torch.cuda.current_stream(src.device)
        for t in temps:
            t.record_stream(cur)


class Bucket:
    __slots__ = ("idx", "lo", "hi", "needed", "filled", "launched", "work", "part_lo", "part_hi",
                 "shard_lo", "shard_len", "event", "agevent", "sparse", "post")

    def __init__(self, idx, lo, hi, needed):
        self.idx, self.lo, self.hi, self.needed = idx, lo, hi, needed
        self.filled = 0
        self.launched = False
        self.work = None
        self.part_lo = self.part_hi = 0
        self.shard_lo = 0     # offset of this bucket's shard in the rank-local shard buffers
        self.shard_len = 0    # elements per rank
        self.event = None     # launching stream: the bucket's last gradient kernel is enqueued
        self.agevent = None   # single-stream mode: after the bucket's parameter all-gather (ZeRO-1)
        self.sparse = False   # reduced by the sparse embedding exchange, not a bucket collective
        self.post = None      # fp32 reduce: copies the reduced fp32 result back (after work.wait())

    @property
    def numel(self):
        return self.hi - self.lo


def make_buckets(flat: FlatParamSpace, bucket_mb: float, solo=()) -> List[Bucket]:
    """Cut the flat buffer into ~bucket_mb ranges at slot boundaries, highest address first.
    Slots named in ``solo`` get a bucket of their own."""
    es = flat.grads.element_size()
    cap = max(1, int(bucket_mb * (1 << 20) / es))
    slots = sorted(flat.slots.values(), key=lambda s: s.offset, reverse=True)
    solo = set(solo)
    out: List[Bucket] = []
    hi = flat.numel
    needed = 0
    for s in slots:
        if s.name in solo:
            if needed:  # close the bucket above the solo slot
                out.append(Bucket(len(out), s.offset + s.numel, hi, needed))
                hi, needed = s.offset + s.numel, 0
            out.append(Bucket(len(out), s.offset, hi, s.numel))
            hi = s.offset
            continue
        needed += s.numel
        if hi - s.offset >= cap:
            out.append(Bucket(len(out), s.offset, hi, needed))
            hi, needed = s.offset, 0
    if needed or hi > 0:
        out.append(Bucket(len(out), 0, hi, needed))
    return out


class GradReducer:
    def __init__(self, flat: FlatParamSpace, extra_sinks: List[GradSink], bucket_mb: Optional[float] = None,
                 mode: Optional[str] = None, group=None, overlap: Optional[bool] = None,
                 sparse_embedding: bool = True, reduce_dtype: str = "native"):
        """``reduce_dtype``: "native" (or "bf16") reduces the gradient buckets in their own
        dtype — RCCL adds in fp32 per hop and rounds to bf16 (tests/test_dp_bf16_numerics.py
        bounds the result); "fp32" (opt-in, ``--dp-reduce-dtype fp32``) reduces an fp32 copy
        of each bucket (2x the bytes on the links) and rounds once at the end."""
        if reduce_dtype not in ("native", "bf16", "fp32"):
            raise ValueError(f"reduce_dtype {reduce_dtype!r}")
        self.reduce_fp32 = reduce_dtype == "fp32" and flat.grads.dtype != torch.float32
        self.flat = flat
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        explicit = mode is not None
        if mode is None:
            mode = "local" if self.world == 1 else "zero1"
        if mode not in MODES:
            raise ValueError(f"unknown gradient mode {mode!r}")
        if self.world == 1 and not (explicit and dist.is_initialized()):
            mode = "local"  # (an explicit mode on a 1-rank process group exercises the collective path)
        if mode == "zero1" and flat.align % (8 * self.world):
            mode = "allreduce"  # shards must stay 8-element aligned for the vector kernels
        self.mode = mode
        self.cuda = flat.device.type == "cuda"
        # Sparse embedding exchange (DP): the token-embedding gradient has at most B*S nonzero
        # rows per rank (2048 of 131072 for Llama-3-8B), yet reducing it densely moves 1 GB per
        # step at the very end of backward, right on the critical path into the next forward.
        # Instead the embedding backward all-gathers the (token, dY row) pairs of every rank
        # (16 MB each) and scatter-adds them locally: every rank gets the full, summed
        # embedding gradient; its bucket needs no collective.
        emb = "tok_embeddings.weight"
        self.sparse_embedding = (sparse_embedding and self.world > 1 and mode != "local" and emb in flat.slots)
        # The token-embedding table in a bucket of its own on one GPU too, so the next forward
        # (which needs it first) waits only for the table's AdamW, not for the layers bucketed
        # with it: GPT-2-medium 15.07 -> 14.97 ms/step, GPT-2-small and 8B unchanged
        # (profiles/r2_emb_solo_bucket_ab.log; FT_EMB_SOLO_BUCKET=0 restores the plain cut)
        solo_emb = self.sparse_embedding or (os.environ.get("FT_EMB_SOLO_BUCKET", "1") == "1" and emb in flat.slots)
        if bucket_mb is None:
            # one GPU: buckets are only the optimizer's launch / gating unit -- finer gating lets the
            # next forward start each layer sooner (8B step 98.4 -> 97.0-97.2 ms from 256 to 16-64 MiB,
            # profiles/r5_bucket_size.log); under DP they are the collectives' size (256 MiB: the
            # xGMI chunk arithmetic in docs/PERFORMANCE.md)
            bucket_mb = LOCAL_BUCKET_MB if mode == "local" else DP_BUCKET_MB
        self.buckets = make_buckets(flat, bucket_mb, solo=(emb,) if solo_emb else ())
        if self.sparse_embedding:
            es = flat.slots[emb]
            for b in self.buckets:
                if b.lo == es.offset and b.hi == es.offset + es.numel:
                    b.sparse = True
            flat.sinks[emb].gather = self._gather_rows
        self.overlap = self.cuda if overlap is None else (overlap and self.cuda)
        # partial sums of squares: a fixed slice per bucket (or per sink, FUSED_SUMSQ) -> the
        # total is a fixed-order sum, deterministic
        self.fused_sumsq = FUSED_SUMSQ and mode == "local" and native(flat.grads) and self.overlap
        self._sq_sinks: List[GradSink] = []
        self._bucket_sq_sinks: List[List[GradSink]] = [[] for _ in self.buckets]
        p = 0
        if self.fused_sumsq:
            fused = list(extra_sinks)
            covered = [(s.start, s.end) for s in fused]
            plain = [s for s in flat.sinks.values()
                     if not any(lo <= s.start and s.end <= hi for lo, hi in covered)]
            for sink in sorted(fused + plain, key=lambda s: s.start, reverse=True):
                k = sink_partials(sink.end - sink.start, sink.buf.dim(), tuple(sink.buf.shape),
                                  128 if sink.buf.dtype == torch.float32 else 256)
                sink.part = (p, p + k)  # replaced by the tensor slice below
                p += k
                self._sq_sinks.append(sink)
                # the bucket holding the sink's lowest address launches after all of it is written
                for b in self.buckets:
                    if b.lo <= sink.start < b.hi:
                        self._bucket_sq_sinks[b.idx].append(sink)
                        break
        else:
            for b in self.buckets:
                n = b.numel // self.world if mode == "zero1" else b.numel
                k = max(1, min(PARTIALS_PER_BUCKET, (n // 8 + 255) // 256))
                b.part_lo, b.part_hi = p, p + k
                p += k
        self.partials = torch.zeros(p, dtype=torch.float32, device=flat.device)
        self._sq_slices = []
        for sink in self._sq_sinks:
            lo, hi = sink.part
            sink.part = self.partials[lo:hi]
            sink.sq_done = False
            self._sq_slices.append(sink.part)
        self._sq_slice_of = {id(s): t for s, t in zip(self._sq_sinks, self._sq_slices)}
        self.sumsq_total = torch.zeros(1, dtype=torch.float32, device=flat.device)
        # ZeRO-1 shard layout: bucket b's shard for this rank, packed in forward order
        self.shard_numel = 0
        if mode == "zero1":
            for b in sorted(self.buckets, key=lambda b: b.lo):
                b.shard_len = b.numel // self.world
                b.shard_lo = self.shard_numel
                self.shard_numel += b.shard_len
        self.side = torch.cuda.Stream(device=flat.device) if self.overlap else None
        self.comm = self.world > 1 or mode != "local"
        # Single-stream collectives (set by graphs.GraphedStep for the whole-step HIP graph): every
        # data-plane collective is issued BLOCKING (async_op=False) on the side stream, so RCCL runs
        # it on that stream, ordered by events. Captured RCCL collectives spread over more than one
        # stream -- ProcessGroupNCCL's internal stream of the async form plus ours, or two of ours --
        # crash hipStreamEndCapture (SIGSEGV, ROCm 7 / RCCL 2.26: the reduce-scatter in backward
        # plus the parameter all-gather after AdamW, i.e. ZeRO-1), while any number of them on ONE
        # stream, with compute-stream round trips between them, capture and replay correctly
        # (scripts/capture_collectives_probe.py, profiles/r6/capture_collectives_probe.log). Eager
        # steps keep the async form: the collectives overlap the side stream's AdamW launches.
        self.single_stream = False
        if not self.fused_sumsq:  # sinks shared with an earlier reducer: no stale partials
            for sink in list(flat.sinks.values()) + list(extra_sinks):
                sink.part, sink.sq_done = None, False
        if self.cuda:
            for b in self.buckets:
                b.event = torch.cuda.Event()
                b.agevent = torch.cuda.Event()
        self._extra_sinks = list(extra_sinks)
        for sink in list(flat.sinks.values()) + list(extra_sinks):
            sink.hook = self._on_ready
        self._pending_sumsq: List[Bucket] = []
        self._next = 0            # index of the next bucket to launch (in-order launch)
        self.fault_after_buckets = 0  # fault-injection hook: raise after this many launches
        # benchmark only (bench.py exposed-communication estimate): skip every collective so a
        # rank runs the same kernels without waiting on peers; gradients are then rank-local
        self.dry_comm = False
        self.sync = True          # False during the non-final micro-batches of an accumulation
        self.gathered = False     # the sparse embedding exchange of this step has run
        self.emb_sink = flat.sinks.get(emb) if self.sparse_embedding else None

    # ---------------------------------------------------------------- shard views
    def param_shard(self, b: Bucket) -> torch.Tensor:
        lo = b.lo + self.rank * b.shard_len
        return self.flat.params[lo : lo + b.shard_len]

    def grad_shard(self, b: Bucket) -> torch.Tensor:
        """This rank's 1/W of bucket b's gradient: the in-place reduce-scatter's output (RCCL
        runs it in place when the output is the rank's own chunk of the input — no separate
        shard buffer, no local copy of that chunk)."""
        lo = b.lo + self.rank * b.shard_len
        return self.flat.grads[lo : lo + b.shard_len]

    def grad_for_update(self, b: Bucket) -> torch.Tensor:
        if self.mode == "zero1":
            # sparse bucket: the full (already summed) gradient is replicated; the rank's slice
            return self.grad_shard(b)
        return self.flat.grads[b.lo : b.hi]

    def _gather_rows(self, tokens: torch.Tensor, dy: torch.Tensor):
        """All-gather every rank's (tokens [T], dY [T, D]) — rank order, deterministic."""
        self.gathered = True
        t = tokens.reshape(-1).contiguous()
        d = dy.reshape(t.numel(), -1).contiguous()
        if self.dry_comm:
            return t, d
        t_all = torch.empty(self.world * t.numel(), dtype=t.dtype, device=t.device)
        d_all = torch.empty(self.world * d.shape[0], d.shape[1], dtype=d.dtype, device=d.device)
        if self.single_stream and self.overlap:  # on the side stream with every other collective
            cur = torch.cuda.current_stream()
            self.side.wait_stream(cur)
            with torch.cuda.stream(self.side):
                dist.all_gather_into_tensor(t_all, t, group=self.group)
                dist.all_gather_into_tensor(d_all, d, group=self.group)
            cur.wait_stream(self.side)
            for x in (t, d, t_all, d_all):
                x.record_stream(self.side)
            return t_all, d_all
        dist.all_gather_into_tensor(t_all, t, group=self.group)
        dist.all_gather_into_tensor(d_all, d, group=self.group)
        return t_all, d_all

    def param_for_update(self, b: Bucket) -> torch.Tensor:
        return self.param_shard(b) if self.mode == "zero1" else self.flat.params[b.lo : b.hi]

    def state_range(self, b: Bucket):
        """(lo, hi) of bucket b in the optimizer-state buffers of this rank."""
        if self.mode == "zero1":
            return b.shard_lo, b.shard_lo + b.shard_len
        return b.lo, b.hi

    # ---------------------------------------------------------------- backward hooks
    def begin_micro(self, k: int, n: int) -> None:
        """Micro-batch ``k`` of ``n`` (gradient accumulation) is about to run forward/backward."""
        last = k == n - 1
        self.sync = last
        for sink in self.flat.sinks.values():
            sink.accumulate = k > 0
        for sink in self._extra_sinks:
            sink.accumulate = k > 0
        for sink in self._sq_sinks:
            sink.sq_done = False  # set again by the producers of this micro-batch
        if self.emb_sink is not None:
            # the sparse exchange sums every rank's rows of every micro-batch at once (in the
            # last backward), so the dense embedding gradient is written once, not accumulated
            self.emb_sink.accumulate = False
            self.emb_sink.defer = not last
            if k == 0:
                self.emb_sink.stash = []

    def _on_ready(self, sink: GradSink) -> None:
        if not self.sync:
            return  # accumulation micro-batch: no collectives, no sums yet
        for b in self.buckets[self._next:]:
            if b.hi <= sink.start:
                break  # buckets are in descending address order
            ov = min(b.hi, sink.end) - max(b.lo, sink.start)
            if ov > 0:
                b.filled += ov
        while self._next < len(self.buckets):
            b = self.buckets[self._next]
            if b.filled < b.needed:
                break
            self._next += 1
            self._launch(b)
            if self.fault_after_buckets and self._next >= self.fault_after_buckets:
                self.fault_after_buckets = 0  # test hook (trainer FT_INJECT_FAULT=r:s:backward)
                raise OSError(5, "injected I/O error inside backward (after a bucket launch)")

    def set_producer_sums(self, on: bool) -> None:
        """A/B switch (scripts/ab_step.py): the gradient producers write the norm partials (on) or
        every sink gets the separate sum-of-squares pass (off). Fused-sumsq reducers only."""
        for sink, part in zip(self._sq_sinks, self._sq_slices):
            sink.part = part if on else None
            sink.sq_done = False

    def _sumsq(self, g: torch.Tensor, b: Bucket) -> None:
        if self.fused_sumsq:
            # per sink: only gradients whose producer did not write its partials this step. Runs of
            # such sinks adjacent in the flat buffer, whose partial slices are adjacent too (slices
            # are assigned in descending address order), take one launch over the whole run: the
            # small models (no producer partials) issued one tiny sumsq kernel per weight
            todo = [sk for sk in self._bucket_sq_sinks[b.idx] if not sk.sq_done]
            for sink in self._bucket_sq_sinks[b.idx]:
                sink.sq_done = False
            grads = self.flat.grads
            base = self.partials.storage_offset()
            runs = []  # [lo, hi, p_lo, p_hi]
            for sk in sorted(todo, key=lambda x: x.start):
                sl = self._sq_slice_of[id(sk)]
                plo = sl.storage_offset() - base
                phi = plo + sl.numel()
                flat_view = sk.buf.data_ptr() == grads.data_ptr() + sk.start * grads.element_size()
                if (runs and flat_view and runs[-1][1] == sk.start and runs[-1][2] == phi
                        and runs[-1][3] - plo <= 65535 and runs[-1][4]):
                    runs[-1][1], runs[-1][2] = sk.end, plo
                else:
                    runs.append([sk.start, sk.end, plo, phi, flat_view, sk])
            for lo, hi, plo, phi, fv, sk in runs:
                if fv:
                    kernels().sumsq_into_(grads[lo:hi], self.partials[plo:phi])
                else:
                    kernels().sumsq_into_(sk.buf.reshape(-1), self._sq_slice_of[id(sk)])
            return
        part = self.partials[b.part_lo : b.part_hi]
        if native(g):
            kernels().sumsq_into_(g, part)
        else:
            part.zero_()
            part[0] = (g.double() if g.dtype == torch.float64 else g.float()).pow(2).sum()

    def _launch(self, b: Bucket) -> None:
        if self.cuda:
            from ..ops.functional import active_dw_stream

            dws = active_dw_stream(self.flat.device)
            if dws is not None and dws != torch.cuda.current_stream():
                # part of this bucket's gradients may still be running on the dW side stream:
                # issue the bucket's work from that stream, after the compute stream's work
                dws.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(dws):
                    self._launch_now(b)
                return
        self._launch_now(b)

    def _collective_blocking(self, b: Bucket, grads: torch.Tensor) -> None:
        """Bucket b's reduction issued blocking on the current (comm) stream: RCCL runs it there."""
        if self.reduce_fp32:
            src = grads.float()
            if self.mode == "allreduce":
                dist.all_reduce(src, op=dist.ReduceOp.SUM, group=self.group)
                grads.copy_(src)
            else:
                out = src.new_empty(b.shard_len)
                dist.reduce_scatter_tensor(out, src, op=dist.ReduceOp.SUM, group=self.group)
                self.grad_shard(b).copy_(out)
        elif self.mode == "allreduce":
            dist.all_reduce(grads, op=dist.ReduceOp.SUM, group=self.group)
        elif self.mode == "zero1":
            dist.reduce_scatter_tensor(self.grad_shard(b), grads, op=dist.ReduceOp.SUM, group=self.group)

    def _launch_now(self, b: Bucket) -> None:
        b.launched = True
        grads = self.flat.grads[b.lo : b.hi]
        if self.single_stream and self.overlap:
            # whole-step graph: the side stream waits for the bucket, reduces it (blocking: RCCL runs
            # on the side stream) and takes its sum of squares; the host never waits
            side = self.side
            b.event.record()
            side.wait_event(b.event)
            with torch.cuda.stream(side):
                if not (b.sparse or self.dry_comm):
                    self._collective_blocking(b, grads)
                if SUMSQ_AT_END:
                    self._pending_sumsq.append(b)
                else:
                    self._sumsq(self.grad_for_update(b), b)
            return
        if b.sparse or self.dry_comm:
            pass  # sparse: summed by the embedding exchange inside the embedding backward
        elif self.reduce_fp32:
            src = grads.float()
            if self.mode == "allreduce":
                b.work = dist.all_reduce(src, op=dist.ReduceOp.SUM, group=self.group, async_op=True)
                b.post = lambda: _copy_back(grads, src, (src,))
            else:
                out = src.new_empty(b.shard_len)
                b.work = dist.reduce_scatter_tensor(out, src, op=dist.ReduceOp.SUM, group=self.group,
                                                    async_op=True)
                shard = self.grad_shard(b)
                b.post = lambda: _copy_back(shard, out, (src, out))
        elif self.mode == "allreduce":
            b.work = dist.all_reduce(grads, op=dist.ReduceOp.SUM, group=self.group, async_op=True)
        elif self.mode == "zero1":
            b.work = dist.reduce_scatter_tensor(self.grad_shard(b), grads, op=dist.ReduceOp.SUM,
                                                group=self.group, async_op=True)
        if not self.overlap:
            return  # CPU / no side stream: sums are taken in finish()
        side = self.side
        if b.work is None:
            b.event.record()  # on the compute stream, after the bucket's last gradient kernel
            side.wait_event(b.event)
        with torch.cuda.stream(side):
            if b.work is not None:
                b.work.wait()  # side stream waits for the collective (host does not)
                b.work = None
                self._post(b)
            if SUMSQ_AT_END:
                self._pending_sumsq.append(b)
            else:
                self._sumsq(self.grad_for_update(b), b)

    @staticmethod
    def _post(b: Bucket) -> None:
        if b.post is not None:
            b.post()
            b.post = None

    def finish(self) -> None:
        """Launch stragglers; after this, ``partials`` hold every bucket's sum of squares
        (on the side stream when overlapping, else synchronously)."""
        if self.cuda:
            from ..ops.functional import join_dw_stream

            join_dw_stream()  # weight gradients still running on the dW side stream
        while self._next < len(self.buckets):
            b = self.buckets[self._next]
            self._next += 1
            self._launch(b)
        if self._pending_sumsq:  # A/B mode: all partial sums after backward, one pass
            with torch.cuda.stream(self.side):
                for b in self._pending_sumsq:
                    self._sumsq(self.grad_for_update(b), b)
            self._pending_sumsq = []
        if not self.overlap:
            for b in self.buckets:
                if b.work is not None:
                    b.work.wait()
                    b.work = None
                    self._post(b)
                self._sumsq(self.grad_for_update(b), b)
        for b in self.buckets:
            b.filled = 0
            b.launched = False
        self._next = 0
        self.gathered = False

    @torch.no_grad()
    def poison_and_complete(self, tokens_shape=None, dim: int = 0) -> None:
        """Finish this rank's share of the step's collectives after a local failure.

        Peers that are still inside the step wait for this rank's remaining bucket
        collectives (and the sparse embedding exchange). Every bucket not yet launched is
        filled with NaN and launched in the usual order, so the peers' collectives complete
        and the reduced gradient — hence the global norm — is NaN on every rank: the
        non-finite guard then skips this step's update everywhere and all ranks keep the
        parameters/moments of the previous step (see ``FlatAdamW.first_nonfinite``).
        Afterwards the caller runs ``optimizer.step()`` as usual (ZeRO-1's norm all-reduce
        and parameter all-gathers are collectives too)."""
        self.sync = True
        nan = float("nan")
        poisoned = False
        for b in self.buckets[self._next:]:
            self.flat.grads[b.lo : b.hi].fill_(nan)
            poisoned = True
        # the peers' order: every dense bucket (they all complete before the embedding
        # backward), then the sparse embedding exchange, then the embedding bucket
        while self._next < len(self.buckets) and not self.buckets[self._next].sparse:
            b = self.buckets[self._next]
            self._next += 1
            self._launch(b)
        if self.sparse_embedding and not self.gathered:
            T = 1
            for s_ in tokens_shape or (1,):
                T *= int(s_)
            tok = torch.zeros(T, dtype=torch.long, device=self.flat.device)
            dy = torch.full((T, dim), nan, dtype=self.flat.dtype, device=self.flat.device)
            self._gather_rows(tok, dy)
            es = self.emb_sink
            self.flat.grads[es.start : es.end].fill_(nan)
            poisoned = True
        # (nothing poisoned: every collective already went out with valid data, so the
        # peers' step — and this rank's, once the caller runs the optimizer — is valid)
        del poisoned
        self.finish()

    def global_sumsq(self) -> torch.Tensor:
        """Partials reduced across ranks when each rank only holds a shard (ZeRO-1).

        Must run on the stream that owns ``partials`` (side stream when overlapping)."""
        if self.mode != "zero1":
            return self.partials
        if self.cuda:
            torch.sum(self.partials, dim=0, keepdim=True, out=self.sumsq_total)
        else:
            self.sumsq_total.copy_(self.partials.sum().reshape(1))
        if not self.dry_comm:
            dist.all_reduce(self.sumsq_total, op=dist.ReduceOp.SUM, group=self.group)
        return self.sumsq_total

    @torch.no_grad()
    def broadcast_params(self, src: int = 0) -> None:
        if self.comm:
            dist.broadcast(self.flat.params, src=src, group=self.group)

    def summary(self) -> str:
        es = self.flat.grads.element_size()
        sizes = [b.numel * es / 2**20 for b in self.buckets]
        return (f"{self.mode}: {len(self.buckets)} buckets, {min(sizes):.0f}-{max(sizes):.0f} MiB"
                + (f", shard {self.shard_numel * es / 2**30:.2f} GiB/rank" if self.mode == "zero1" else ""))

