"""Autograd functions of the transformer hot path.

GPU tensors run the hand-written gfx950 kernels in ``csrc/kernels`` (loaded by
:func:`fault_tolerant_llm_training_amd._native.kernels`, which raises if the
library is missing) and hipBLASLt GEMMs through ``torch.mm``/``torch.addmm``.
Model dtypes (``--model-dtype``): bf16 (every kernel), fp16 (every kernel; the MFMA GEMM and
flash kernels in their fp16 variants), fp32 (the element-wise / reduction kernels in fp32,
fp32 attention kernels, fp32 hipBLASLt GEMMs; the bf16-only paths — the round-2 hand GEMM, the
transpose-based weight gradients, the fused SwiGLU transposes — route by dtype).
CPU tensors run a pure-PyTorch reference of the same math (the CPU backend for
the gloo tests); its backward recomputes the forward under autograd.

Weight gradients never go through ``AccumulateGrad``: each function writes
them into the parameter's :class:`GradSink` (a view of the flat gradient
buffer) and returns ``None`` for the weight.

Reference parity (math): RMSNorm model.py:24-48, RoPE model.py:100-126,
attention model.py:179-215, SwiGLU model.py:253-254, embedding model.py:373,
LM head model.py:379, loss train.py:101-102.
"""
from __future__ import annotations

import collections
import functools
import os
from typing import Optional

import torch
import torch.nn.functional as F

from .._native import kernels, native
from .grad_sink import GradSink

IGNORE_INDEX = -100

# GEMM backend per product: the hand-written gfx950 kernel (csrc/kernels/gemm.hip) reads every
# operand in its row-major layout (no transposes) and fuses SwiGLU into the FFN GEMMs;
# hipBLASLt (torch.mm) is kept where it measures faster. FT_GEMM = "auto" (per-product policy
# below, from scripts/gemm_bench.py on MI355X), "hand" (every fitting shape), "blas" (none).
_GEMM_MODE = os.environ.get("FT_GEMM", "auto")
# products the hand kernel takes in "auto" (FT_GEMM_AUTO, comma list of fwd,dx,dw,ffn).
# Default: none. Measured on the Llama-3-8B step (profiles/r2_gemm_hand_vs_hipblaslt.md,
# profiles/r2_gemm_asm_reads_ab.log): the hand kernel runs the products at 0.56-1.06x of
# hipBLASLt, and the whole step at 109.4 ms (all hipBLASLt) vs 112.9 (SwiGLU-fused FFN on the
# hand kernel), 118.8 (FFN + dW), 123.1 (every product); after the asm-read fix, hand dX 0.989x
# and hand dW 0.963x of the all-hipBLASLt step — the transposes and SwiGLU passes it removes
# cost less than the GEMM speed it gives up.
_HAND_AUTO = set(k for k in os.environ.get("FT_GEMM_AUTO", "").split(",") if k)


def _parse_shapes(spec: str):
    """"dw:4096x14336x2048,dx:..." -> {("dw", 4096, 14336, 2048), ...} (kind, M, N, K of _hand)."""
    out = set()
    for item in (x for x in spec.split(",") if x):
        kind, dims = item.split(":")
        m, n, k = (int(v) for v in dims.lower().split("x"))
        out.add((kind, m, n, k))
    return out


# Individual products the hand kernel takes in "auto" (FT_GEMM_HAND_SHAPES, kind:MxNxK list;
# "" for none). Default: the Llama-3-8B weight gradient of wo, where the hand kernel (asm
# fragment reads, row-major dY / X read in place) beats hipBLASLt alone (69.0 vs 72.8 us) and
# ties it in the step (109.16 vs 109.06 ms, same-process A/B). w2's dW from the SwiGLU
# kernels' a^T (no transposes at all) measured 0.996x in the step, so it stays opt-in
# ("dw:4096x14336x2048"); profiles/r2_gemm_hand_dw_wo_w2_ab.log.
_HAND_SHAPES = _parse_shapes(os.environ.get("FT_GEMM_HAND_SHAPES", "dw:4096x4096x2048"))


def set_gemm_mode(mode: str) -> None:
    global _GEMM_MODE
    if mode not in ("auto", "hand", "blas"):
        raise ValueError(mode)
    _GEMM_MODE = mode


def _hand(kind: str, M: int, N: int, K: int, *ts) -> bool:
    """Use the hand GEMM for product ``kind`` ("fwd", "dx", "dw", "ffn") of shape M x N x K?"""
    if _GEMM_MODE == "blas" or not all(t.is_cuda and t.dtype == torch.bfloat16 for t in ts):
        return False
    if M % 128 or N % 128 or K % 64:  # 256 x 256 tiles where they fill the chip, else 128 x 128
        return False
    if _GEMM_MODE == "hand" or kind in _HAND_AUTO or (kind, M, N, K) in _HAND_SHAPES:
        return True
    # tall-K product with few 256x256 output tiles (the LM head's dX for GPT-2-sized models,
    # [2048 x 768 x 131072]): the hand kernel's split-K fills the chip where hipBLASLt does not
    # (496 vs 722 us at d=768, 570 vs 889 us at d=1024; profiles/r2_gemm_gpt2_shapes.log)
    return kind == "dx" and (M // 256) * (N // 256) < 64 and K >= 16384


# GEMMs on the 4-wave hand kernel (csrc/kernels/gemm_w4.hip), K-contiguous operands (x W^T):
#   FT_W4_FWD    (default on) forward products whose tile width is narrower than 256 (it fills the
#                256 CUs in whole rounds where the 256-wide vendor tiles leave a partial round:
#                Llama-3-8B qkv 1.14x, wo 1.09x, w2 1.02x of hipBLASLt; w13 / LM head stay on it)
#   FT_W4_DW=1   weight gradients dW = dY^T X on the transposed operands (every size)
_W4_FWD = os.environ.get("FT_W4_FWD", "1") != "0"
_W4_DW = os.environ.get("FT_W4_DW", "0") == "1"
_W4_FWD_MAX_NJ = int(os.environ.get("FT_W4_FWD_MAX_NJ", "6"))


def set_w4_fwd(on: bool) -> None:
    global _W4_FWD
    _W4_FWD = bool(on)


def set_w4_dw(on: bool) -> None:
    global _W4_DW
    _W4_DW = bool(on)


_W4_DTYPES = (torch.bfloat16, torch.float16)  # bf16 / fp16 MFMA variants of the kernel
# Output tiles (of 256 rows) a product needs before it goes to the w4 kernel: half the chip.
# (Tests lower it to drive small shapes through the same paths.)
_W4_MIN_TILES = 128


def _w4_fits(x2: torch.Tensor, w: torch.Tensor, max_nj: int = 8) -> bool:
    if _GEMM_MODE == "blas" or not (x2.is_cuda and x2.dtype in _W4_DTYPES and w.dtype == x2.dtype):
        return False
    T, K = x2.shape
    if T % 256 or K % 128:  # the w4 kernel runs K-tiles of 64 in pairs
        return False
    nj = kernels().gemm_w4_pick(T, w.shape[0])
    # at least half the chip in tiles: smaller products (GPT-2-sized, K = 768-1024) are
    # latency-bound and stay on the vendor kernels
    return 0 < nj <= max_nj and (T // 256) * (w.shape[0] // (32 * nj)) >= _W4_MIN_TILES


def _w4_ok(x2: torch.Tensor, w: torch.Tensor) -> bool:
    return _W4_FWD and _w4_fits(x2, w, _W4_FWD_MAX_NJ)


# GPT-2-sized forward products on the 128 x 128-tile kernel (csrc/kernels/gemm_s.hip): K <= 1024
# and at least 256 output tiles. Alone (graph-timed) it runs GPT-2-small qkv 1.20x / w13 1.10x,
# -medium qkv 1.05x / w13 1.15x hipBLASLt (profiles/r3_gemm_s_vs_hipblaslt.log), but inside the
# graph-replayed step it measured 0.99-1.00x (its two workgroups per CU share the CUs with the
# pipelined optimizer and the dW stream; profiles/r3_gpt2_s_ab.log): opt-in, FT_GEMM_S=1.
_GEMM_S = os.environ.get("FT_GEMM_S", "0") == "1"


def set_gemm_s(on: bool) -> None:
    global _GEMM_S
    _GEMM_S = bool(on)


def _s_ok(x2: torch.Tensor, w: torch.Tensor) -> bool:
    if not (_GEMM_S and _GEMM_MODE != "blas" and x2.is_cuda and x2.dtype in _W4_DTYPES and w.dtype == x2.dtype):
        return False
    T, K = x2.shape
    N = w.shape[0]
    return T % 128 == 0 and N % 128 == 0 and K % 64 == 0 and K <= 1024 and (T // 128) * (N // 128) >= 256


def mm_fwd(x2: torch.Tensor, w: torch.Tensor, residual: Optional[torch.Tensor] = None) -> torch.Tensor:
    """y = x2 @ w^T (+ residual): x2 [T, K], w [N, K] (nn.Linear layout)."""
    T, K = x2.shape
    N = w.shape[0]
    if _s_ok(x2, w):
        return kernels().gemm_nt_s(x2.contiguous(), w, None,
                                   None if residual is None else residual.reshape(T, N).contiguous(), 1)
    if _w4_ok(x2, w):
        return kernels().gemm_nt_w4(x2.contiguous(), w, None,
                                    None if residual is None else residual.reshape(T, N).contiguous(), 0)
    if _hand("fwd", T, N, K, x2, w):
        return kernels().gemm(x2.contiguous(), True, w, True, T, N, K, None,
                              None if residual is None else residual.reshape(T, N).contiguous(), False, 0)
    if residual is None:
        return torch.mm(x2, w.t())
    return torch.addmm(residual.reshape(T, N), x2, w.t())


# Backward GEMMs on the w4 kernel's k-major layouts (csrc/kernels/gemm_w4.hip, gemm_w4_ex): dX = dY W
# reads the weight [N, K] as stored, dW = dY^T X reads dY [T, N] and X [T, K] as stored, through
# ds_read_b64_tr_b16 transposed LDS reads -- no transposed copies, no transpose kernel. The dW
# epilogue also writes the gradient's per-tile sums of squares into the sink's norm partials (one
# GPU), so no separate pass re-reads the gradient for clip_grad_norm_. Default on; FT_W4_BWD=0
# restores the round-3 routing (hipBLASLt, transposed copies for dW) for A/B runs.
_W4_BWD = os.environ.get("FT_W4_BWD", "1") != "0"


def set_w4_bwd(on: bool) -> None:
    global _W4_BWD
    _W4_BWD = bool(on)


def _w4t_fits(M: int, N: int, K: int, *ts) -> bool:
    """C[M, N] over a K-deep sum on the w4 kernel: 16-bit CUDA operands of one dtype, a tile width
    for N, and at least half the chip in tiles (smaller, GPT-2-sized products are latency-bound
    and stay on the vendor kernels)."""
    if not (_W4_BWD and _GEMM_MODE != "blas" and all(t.is_cuda and t.dtype in _W4_DTYPES for t in ts)
            and len({t.dtype for t in ts}) == 1):
        return False
    if M % 256 or K % 128 or K < 128:  # K-tiles of 64 in pairs
        return False
    nj = kernels().gemm_w4_pick(M, N)
    return 0 < nj and (M // 256) * (N // (32 * nj)) >= _W4_MIN_TILES


# dX products with a deep reduction (N >= 16384: the 8B w13 dX, N = 2F = 28672, and the LM-head
# dX, N = V) whose 256-wide tiles fill only half the chip run split-K on the w4 kernel (each tile's
# two K halves on two workgroups, gemm_w4.h): with 256 x 128 tiles instead the loop is LDS-bound
# (0.88-0.90x of hipBLASLt, profiles/r4_gemm_w4t_bench.log). Without a split (FT_W4_SPLITK=0)
# they go back to hipBLASLt.
_W4_DX_DEEP_K = 16384


@functools.lru_cache(maxsize=256)
def _w4_plan(M: int, N: int, K: int, a_t: bool, b_t: bool):
    """(tile width / 32, splits) of the w4 kernel's automatic plan for C[M, N] over K."""
    return tuple(kernels().gemm_w4_plan(M, N, K, a_t, b_t))


def set_w4_splitk(mode: int) -> None:
    """Split-K of the w4 kernel (FT_W4_SPLITK): 0 off, 1 automatic (default), 2 forced where it fits."""
    kernels().gemm_w4_set_splitk(int(mode))
    _w4_plan.cache_clear()


def _w4_dx_ok(T: int, K: int, N: int, dy2: torch.Tensor, w: torch.Tensor) -> bool:
    if not (_w4t_fits(T, K, N, dy2, w) and w.is_contiguous()):
        return False
    if N >= _W4_DX_DEEP_K and (T // 256) * (K // 256) <= 256:
        return _w4_plan(T, K, N, False, True)[1] > 1
    return True


def mm_dx(dy2: torch.Tensor, w: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """dx = dy2 @ w: dy2 [T, N], w [N, K]."""
    T, N = dy2.shape
    K = w.shape[1]
    if _w4_dx_ok(T, K, N, dy2, w):
        return kernels().gemm_w4_ex(dy2.contiguous(), False, w, True, T, K, N, out, False, None, 0)
    if out is not None:
        if _hand("dx", T, K, N, dy2, w):
            return kernels().gemm(dy2.contiguous(), True, w, False, T, K, N, out, None, False, 0)
        return torch.mm(dy2, w, out=out)
    if _hand("dx", T, K, N, dy2, w):
        return kernels().gemm(dy2.contiguous(), True, w, False, T, K, N, None, None, False, 0)
    return torch.mm(dy2, w)

# Weight gradients dW = dY^T X as a K-contiguous ("TN") GEMM on transposed copies of
# both operands: hipBLASLt runs that layout ~1.3x faster on MI355X than the
# token-major ("NT") product of the row-major activations, and the gfx950
# transpose kernel costs far less than the difference for the large projections
# (scripts/gemm_layout_bench.py). FT_DW_TRANSPOSE: "auto" (default, big GEMMs only),
# "all", "none".
_DW_MODE = os.environ.get("FT_DW_TRANSPOSE", "auto")
_DW_MIN_FLOP = 2.0e11


def _use_tn(dy2: torch.Tensor, x2: torch.Tensor) -> bool:
    if _DW_MODE == "none" or not dy2.is_cuda or dy2.dtype != torch.bfloat16:
        return False
    T, N = dy2.shape
    K = x2.shape[1]
    if T % 64 or N % 64 or K % 64:
        return False
    if _W4_DW and T % 128 == 0 and N % 256 == 0 and kernels().gemm_w4_pick(N, K) > 0:
        return True  # the w4 kernel runs dW on the transposed (K-contiguous) operands
    return _DW_MODE == "all" or 2.0 * T * N * K >= _DW_MIN_FLOP


def weight_grad(dy2: torch.Tensor, x2: torch.Tensor, sink: Optional[GradSink],
                dyT: Optional[torch.Tensor] = None, xT: Optional[torch.Tensor] = None, bufs=None):
    """dW[N, K] = dy2[T, N]^T @ x2[T, K], into the sink (flat grad buffer) or returned.

    ``dyT`` / ``xT``: already-transposed operands written by a producer kernel (the fused
    SwiGLU kernels), used instead of running the transpose kernel. ``x2`` may then be None.
    ``bufs``: preallocated (dyT, xT) outputs for the transposes (see weight_grad_async)."""
    if xT is not None and x2 is None:
        x2 = xT.t()
    T, N = dy2.shape
    K = x2.shape[1]
    if dyT is None and xT is None and _w4t_fits(N, K, T, dy2, x2) and dy2.is_contiguous() and x2.is_contiguous():
        # dW[N, K] = dY^T X, both read as stored (k-major A and B), straight into the sink
        if sink is None:
            return kernels().gemm_w4_ex(dy2, True, x2, True, N, K, T, None, False, None, 0)
        kernels().gemm_w4_ex(dy2, True, x2, True, N, K, T, sink.buf.view(N, K), sink.accumulate, sink.part, 0)
        if sink.part is not None:
            sink.sq_done = True
        sink.ready()
        return None
    if xT is not None and dyT is None and _hand("dw", N, K, T, dy2, xT) and dy2.is_contiguous() \
            and xT.is_contiguous():
        # dW[N, K] = dY^T X with X given transposed (the SwiGLU kernels' a^T [K, T]): the hand
        # kernel reads dY [T, N] as A^T and X^T as a K-contiguous B — no transposes at all
        out = sink.buf.view(N, K) if sink is not None else None
        acc = sink.accumulate if sink is not None else False
        r = kernels().gemm(dy2, False, xT, True, N, K, T, out, None, acc, 0)
        if sink is not None:
            sink.ready()
            return None
        return r
    if _hand("dw", N, K, T, dy2, x2) and dy2.is_contiguous() and x2.is_contiguous():
        # dW[N, K] = dY^T X read straight from the row-major dY [T, N] and X [T, K]
        out = sink.buf.view(N, K) if sink is not None else None
        acc = sink.accumulate if sink is not None else False
        r = kernels().gemm(dy2, False, x2, False, N, K, T, out, None, acc, 0)
        if sink is not None:
            sink.ready()
            return None
        return r
    if _use_tn(dy2, x2):
        K_ = kernels()
        ba, bb = bufs if bufs is not None else (None, None)
        a = dyT if dyT is not None else K_.transpose2d(dy2.contiguous(), ba)   # [N, T]
        b = xT if xT is not None else K_.transpose2d(x2.contiguous(), bb)      # [K, T]
        if _W4_DW and _w4_fits(a, b):
            if sink is not None:
                out = sink.buf.view(N, K)
                K_.gemm_nt_w4(a, b, out, out if sink.accumulate else None, 0)
                sink.ready()
                return None
            return K_.gemm_nt_w4(a, b, None, None, 0)
        if sink is not None:
            sink.mm(a, b.t())
            return None
        return torch.mm(a, b.t())
    if sink is not None:
        sink.mm(dy2.t(), x2)
        return None
    return torch.mm(dy2.t(), x2)


# Weight-gradient GEMMs on a side stream (default; FT_DW_STREAM=0 disables): dW and the dX
# GEMM of the same node are independent, and the small projections (wo, wqkv: 128-192
# output tiles of 256x256) leave half of the 256 CUs idle when run one after the other
# (8B step: 108.6 -> 107.1 ms, profiles/r1_dw_stream_ab.log). The side stream
# waits for the compute stream before each dW (so it sees dY / X), the operands are
# recorded on it (the caching allocator keeps them alive), and the bucket hooks fired
# from it order the reducer's collectives after it. join_dw_stream() (GradReducer.finish,
# FlatAdamW.step) makes the compute stream wait for every dW before the optimizer.
_DW_STREAM = os.environ.get("FT_DW_STREAM", "1") == "1"
_dw_streams = {}
_dw_pending = {}  # device -> FIFO of (dW done event, operands kept alive until then)
_DW_LAG = int(os.environ.get("FT_DW_LAG", "4"))  # dW GEMMs the compute stream may run ahead by
# dW GEMMs that take the w4 kernel on k-major operands run inline unless FT_W4_DW_SIDE=1
_W4_DW_SIDE = os.environ.get("FT_W4_DW_SIDE", "0") == "1"


def set_dw_stream(on: bool) -> None:
    global _DW_STREAM
    _DW_STREAM = bool(on)


def _dev_key(dev: torch.device) -> int:
    return dev.index if dev.index is not None else torch.cuda.current_device()


def _dw_side(dev: torch.device) -> torch.cuda.Stream:
    k = _dev_key(dev)
    s = _dw_streams.get(k)
    if s is None:
        s = _dw_streams[k] = torch.cuda.Stream(device=k)
    return s


def weight_grad_async(dy2: torch.Tensor, x2: Optional[torch.Tensor], sink: Optional[GradSink],
                      dyT: Optional[torch.Tensor] = None, xT: Optional[torch.Tensor] = None):
    """:func:`weight_grad` into ``sink`` on the dW side stream (or inline when disabled)."""
    if not (_DW_STREAM and dy2.is_cuda and sink is not None):
        return weight_grad(dy2, x2, sink, dyT, xT)
    cur = torch.cuda.current_stream(dy2.device)
    side = _dw_side(dy2.device)
    # Operand lifetime is stream-ordered instead of record_stream(): the operands (and the
    # transposes' outputs, allocated here on the compute stream) stay referenced in a short
    # FIFO; before one is dropped the compute stream waits for its dW, so the freed blocks
    # are reusable by the compute stream at once. record_stream() kept every recorded
    # activation out of the caching allocator until its event had completed, and with the
    # host a step ahead of the GPU that held HBM at ~1.6x the allocated peak and sent
    # long-context steps into allocator cache flushes (profiles/r1_allocator_pools.log).
    dy2 = dy2.contiguous()
    x2 = x2.contiguous() if x2 is not None else None
    xx = x2 if x2 is not None else xT.t()
    bufs = None
    w4t = dyT is None and xT is None and _w4t_fits(dy2.shape[1], xx.shape[1], dy2.shape[0], dy2, xx)
    if w4t and not _W4_DW_SIDE:
        # the w4 kernels hold one workgroup per CU: a concurrent dX kernel cannot co-reside, so the
        # side stream only adds cross-stream waits (8B step 108.5 -> 106.9 ms with dW inline,
        # profiles/r4_ab.log)
        return weight_grad(dy2, x2, sink, dyT, xT)
    if not w4t and _use_tn(dy2, xx) and not _hand("dw", dy2.shape[1], xx.shape[1], dy2.shape[0], dy2, xx):
        T, N = dy2.shape
        bufs = (dy2.new_empty((N, T)) if dyT is None else None,
                xx.new_empty((xx.shape[1], T)) if xT is None else None)
    side.wait_stream(cur)
    with torch.cuda.stream(side):
        weight_grad(dy2, x2, sink, dyT, xT, bufs)
        ev = torch.cuda.Event()
        ev.record()
    q = _dw_pending.setdefault(_dev_key(dy2.device), collections.deque())
    q.append((ev, (dy2, x2, dyT, xT, bufs)))
    while len(q) > _DW_LAG:
        cur.wait_event(q.popleft()[0])
    return None


def active_dw_stream(dev: torch.device) -> Optional[torch.cuda.Stream]:
    """The dW side stream of ``dev`` if weight gradients may be in flight on it, else None."""
    return _dw_streams.get(_dev_key(dev)) if _DW_STREAM else None


def join_dw_stream() -> None:
    """Make the current stream wait for all weight gradients issued on the dW side stream."""
    if _dw_streams:
        cur = torch.cuda.current_stream()
        k = _dev_key(cur.device)
        s = _dw_streams.get(k)
        if s is not None:
            cur.wait_stream(s)
            q = _dw_pending.get(k)
            if q:
                q.clear()  # every dW is ordered before the compute stream's next work


def norm_bwd_into_sink(dy, x, w, rstd, mean, sink: GradSink, dres=None) -> torch.Tensor:
    """dx of the (add-)norm backward; dW folded into ``sink`` (then ``sink.ready()``), with its
    per-column-block sums of squares into the sink's norm partials when it has them.
    (Folding dW on the dW side stream instead was measured at no gain:
    profiles/r1_norm_fold_side_ab.log.)"""
    dx = kernels().norm_bwd(dy, x, w, rstd, mean, sink.buf, dres, sink.accumulate, sink.part)
    if sink.part is not None:
        sink.sq_done = True
    sink.ready()
    return dx


def _write_weight_grad(sink: Optional[GradSink], g: torch.Tensor):
    """CPU helper: route a computed weight gradient into its sink (or return it)."""
    if sink is None:
        return g
    sink.set_(g.to(sink.buf.dtype))
    return None


# --------------------------------------------------------------------------------------
# Embedding
# --------------------------------------------------------------------------------------
class EmbeddingFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, tokens, weight, sink):
        ctx.sink = sink
        ctx.vocab = weight.shape[0]
        ctx.save_for_backward(tokens)
        ctx.wshape = weight.shape
        if native(weight):
            return kernels().embedding_fwd(tokens.contiguous(), weight)
        return F.embedding(tokens, weight)

    @staticmethod
    def backward(ctx, dy):
        (tokens,) = ctx.saved_tensors
        sink = ctx.sink
        dy = dy.contiguous()
        if sink is not None and sink.gather is not None:
            if sink.defer:  # accumulation micro-batch: exchanged with the last one
                sink.stash.append((tokens.reshape(-1), dy.reshape(-1, dy.shape[-1])))
                return None, None, None
            if sink.stash:
                tokens = torch.cat([t for t, _ in sink.stash] + [tokens.reshape(-1)])
                dy = torch.cat([g for _, g in sink.stash] + [dy.reshape(-1, dy.shape[-1])])
                sink.stash = []
            # DP sparse exchange: every rank's (token, dY) rows, scatter-added locally
            tokens, dy = sink.gather(tokens, dy)
        if native(dy):
            if sink is None:
                dw = torch.zeros(ctx.wshape, dtype=dy.dtype, device=dy.device)
                kernels().embedding_bwd_(dy, tokens.contiguous(), dw, False)
                return None, dw, None
            # a fresh gradient: the kernel also writes the norm partials of the rows it stores (every
            # other row is zero), so the reducer's sum-of-squares pass over the [V, D] buffer is skipped
            part = sink.part if (sink.part is not None and not sink.accumulate) else None
            kernels().embedding_bwd_(dy, tokens.contiguous(), sink.buf, sink.accumulate, part)
            if part is not None:
                sink.sq_done = True
            sink.ready()
            return None, None, None
        dw = torch.zeros(ctx.wshape, dtype=torch.float32, device=dy.device)
        if dy.is_cuda:  # (fp64 models on the GPU) index_add_ is atomic there; the sorted
            # accumulate of index_put_ is deterministic (bit-exact resume)
            dw.index_put_((tokens.reshape(-1),), dy.reshape(-1, ctx.wshape[1]).float(), accumulate=True)
        else:
            dw.index_add_(0, tokens.reshape(-1), dy.reshape(-1, ctx.wshape[1]).float())
        return None, _write_weight_grad(sink, dw.to(dy.dtype)), None


def embedding(tokens, weight, sink=None):
    return EmbeddingFn.apply(tokens, weight, sink)


# --------------------------------------------------------------------------------------
# RMSNorm / LayerNorm (weight only)
# --------------------------------------------------------------------------------------
def norm_reference(x: torch.Tensor, w: torch.Tensor, eps: float, layernorm: bool) -> torch.Tensor:
    xf = x.float()
    if layernorm:
        xf = xf - xf.mean(-1, keepdim=True)
    n = xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps)
    return n.type_as(x) * w


class NormFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, sink, eps, layernorm):
        ctx.sink, ctx.eps, ctx.ln = sink, eps, layernorm
        if native(x):
            xc = x.contiguous()
            y, rstd, mean = kernels().norm_fwd(xc, weight, eps, layernorm)
            ctx.save_for_backward(xc, weight, rstd, mean)
            return y
        ctx.save_for_backward(x, weight)
        return norm_reference(x, weight, eps, layernorm)

    @staticmethod
    def backward(ctx, dy):
        sink = ctx.sink
        if native(dy):
            x, w, rstd, mean = ctx.saved_tensors
            if sink is not None:
                return norm_bwd_into_sink(dy.contiguous(), x, w, rstd, mean, sink), None, None, None, None
            dw = torch.empty_like(w)
            dx = kernels().norm_bwd(dy.contiguous(), x, w, rstd, mean, dw, None, False)
            return dx, dw, None, None, None
        x, w = ctx.saved_tensors
        with torch.enable_grad():
            xr = x.detach().requires_grad_(True)
            wr = w.detach().requires_grad_(True)
            y = norm_reference(xr, wr, ctx.eps, ctx.ln)
            dx, dw = torch.autograd.grad(y, (xr, wr), dy)
        return dx, _write_weight_grad(sink, dw), None, None, None


def norm(x, weight, sink=None, eps: float = 1e-5, layernorm: bool = False):
    return NormFn.apply(x, weight, sink, eps, layernorm)


class AddNormFn(torch.autograd.Function):
    """(h, y) = (x + d, norm(x + d)): the residual add of the previous sub-block fused
    into the next pre-norm (reference model.py:310-311 ``h = x + attn(norm(x))``).

    Backward is one kernel: dh_total = dres + norm_bwd(dy), returned for both x and d.
    """

    @staticmethod
    def forward(ctx, x, d, weight, sink, eps, layernorm):
        ctx.sink, ctx.eps, ctx.ln = sink, eps, layernorm
        if native(x):
            y, rstd, mean, h = kernels().add_norm_fwd(x.contiguous(), d.contiguous(), weight, eps, layernorm)
            ctx.save_for_backward(h, weight, rstd, mean)
            return h, y
        h = x + d
        ctx.save_for_backward(h, weight)
        return h, norm_reference(h, weight, eps, layernorm)

    @staticmethod
    def backward(ctx, dh, dy):
        sink = ctx.sink
        if native(dy):
            h, w, rstd, mean = ctx.saved_tensors
            dres = dh.contiguous() if dh is not None else None
            if sink is not None:
                g = norm_bwd_into_sink(dy.contiguous(), h, w, rstd, mean, sink, dres)
                return g, g, None, None, None, None
            buf = torch.empty_like(w)
            g = kernels().norm_bwd(dy.contiguous(), h, w, rstd, mean, buf, dres, False)
            return g, g, buf, None, None, None
        h, w = ctx.saved_tensors
        with torch.enable_grad():
            hr = h.detach().requires_grad_(True)
            wr = w.detach().requires_grad_(True)
            y = norm_reference(hr, wr, ctx.eps, ctx.ln)
            g, dw = torch.autograd.grad(y, (hr, wr), dy)
        if dh is not None:
            g = g + dh
        return g, g, _write_weight_grad(sink, dw), None, None, None


def add_norm(x, d, weight, sink=None, eps: float = 1e-5, layernorm: bool = False):
    """Returns (x + d, norm(x + d))."""
    return AddNormFn.apply(x, d, weight, sink, eps, layernorm)


# --------------------------------------------------------------------------------------
# Linear (+ fused residual add through the GEMM's C input)
# --------------------------------------------------------------------------------------
class LinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, sink, residual):
        K = x.shape[-1]
        N = weight.shape[0]
        x2 = x.reshape(-1, K)
        y = mm_fwd(x2, weight, residual)
        ctx.sink = sink
        ctx.has_res = residual is not None
        ctx.xshape = x.shape
        ctx.save_for_backward(x2, weight)
        return y.view(*x.shape[:-1], N)

    @staticmethod
    def backward(ctx, dy):
        x2, w = ctx.saved_tensors
        N = w.shape[0]
        dy2 = dy.reshape(-1, N)
        dw = None
        # weight gradient first, so its all-reduce bucket can launch while dx runs
        dw = weight_grad_async(dy2, x2, ctx.sink)
        dx = mm_dx(dy2, w).view(ctx.xshape)
        return dx, dw, None, (dy if ctx.has_res else None)


def linear(x, weight, sink=None, residual=None):
    return LinearFn.apply(x, weight, sink, residual)


# --------------------------------------------------------------------------------------
# RoPE + causal GQA attention on the fused QKV projection
# --------------------------------------------------------------------------------------
def rope_reference(x: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor) -> torch.Tensor:
    """x: [B, S, H, D] interleaved pairs; cos/sin: [S, D/2] fp32."""
    xf = x.float().reshape(*x.shape[:-1], -1, 2)
    a, b = xf[..., 0], xf[..., 1]
    c = cos[: x.shape[1]].view(1, x.shape[1], 1, -1)
    s = sin[: x.shape[1]].view(1, x.shape[1], 1, -1)
    out = torch.stack((a * c - b * s, a * s + b * c), dim=-1).flatten(-2)
    return out.type_as(x)


def attention_reference(qkv, cos, sin, seq_len, hq, hkv, d):
    """Reference math: RoPE → repeat_kv → causal SDPA (model.py:179-215). qkv: [B*S, W]."""
    T = qkv.shape[0]
    B = T // seq_len
    q = qkv[:, : hq * d].reshape(B, seq_len, hq, d)
    k = qkv[:, hq * d : (hq + hkv) * d].reshape(B, seq_len, hkv, d)
    v = qkv[:, (hq + hkv) * d :].reshape(B, seq_len, hkv, d)
    q = rope_reference(q, cos, sin)
    k = rope_reference(k, cos, sin)
    rep = hq // hkv
    if rep > 1:
        k = k.repeat_interleave(rep, dim=2)
        v = v.repeat_interleave(rep, dim=2)
    o = F.scaled_dot_product_attention(q.transpose(1, 2), k.transpose(1, 2), v.transpose(1, 2), is_causal=True)
    return o.transpose(1, 2).reshape(T, hq * d)


class AttentionKeep:
    """Per-block holder of the attention output kept across a recomputed block (selective
    activation checkpointing): the first forward of a checkpointed block stores (o, lse) here
    tagged with the model's forward generation; the recompute in backward (same generation)
    reuses them instead of running the flash forward again. A stale entry (a forward whose
    backward never ran) carries an older generation and is simply overwritten."""

    __slots__ = ("gen", "o", "lse")

    def __init__(self):
        self.gen, self.o, self.lse = -1, None, None


class RopeAttentionFn(torch.autograd.Function):
    """RoPE + causal GQA attention on the packed projection. ``rotated``: Q/K of ``qkv`` were
    already rotated by the QKV projection's epilogue (:class:`QKVRopeFn`, GPU only): the flash
    kernels then read Q/K straight from ``qkv``. Either way backward returns the gradient of the
    UNROTATED projection: the flash backward rotates dQ/dK back in the pass that folds the GQA
    dK/dV partials (so neither this node nor the projection's backward runs a RoPE pass)."""

    @staticmethod
    def forward(ctx, qkv, cos, sin, seq_len, hq, hkv, d, keep=None, gen=-1, rotated=False):
        ctx.cfg = (seq_len, hq, hkv, d)
        ctx.rotated = rotated
        hit = keep is not None and keep.gen == gen and keep.o is not None
        if native(qkv):
            from .attention import flash_attn_fwd

            qkv = qkv.contiguous()
            qk = qkv if rotated else kernels().rope_fwd(qkv, cos, sin, seq_len, hq, hkv, d)
            if hit:  # recompute pass of a checkpointed block: the kept output (bit-identical)
                o, lse = keep.o, keep.lse
                keep.o = keep.lse = None
            else:
                o, lse = flash_attn_fwd(qk, qkv, seq_len, hq, hkv, d)
                if keep is not None:
                    keep.gen, keep.o, keep.lse = gen, o, lse
            ctx.save_for_backward(qkv, qk, o, lse, cos, sin)
            return o
        ctx.save_for_backward(qkv, cos, sin)
        if hit:
            o = keep.o
            keep.o = None
        else:
            o = attention_reference(qkv, cos, sin, seq_len, hq, hkv, d)
            if keep is not None:
                keep.gen, keep.o = gen, o
        return o

    @staticmethod
    def backward(ctx, do):
        seq_len, hq, hkv, d = ctx.cfg
        if native(do):
            from .attention import flash_attn_bwd

            qkv, qk, o, lse, cos, sin = ctx.saved_tensors
            dqkv = flash_attn_bwd(do.contiguous(), qk, qkv, o, lse, seq_len, hq, hkv, d, cos, sin)
            return dqkv, None, None, None, None, None, None, None, None, None
        qkv, cos, sin = ctx.saved_tensors
        with torch.enable_grad():
            x = qkv.detach().requires_grad_(True)
            o = attention_reference(x, cos, sin, seq_len, hq, hkv, d)
            (dx,) = torch.autograd.grad(o, (x,), do)
        return dx, None, None, None, None, None, None, None, None, None


def rope_attention(qkv, cos, sin, seq_len, hq, hkv, d, keep: Optional[AttentionKeep] = None, gen: int = -1,
                   rotated: bool = False):
    """RoPE on the packed projection, then causal GQA attention. ``keep``/``gen``: selective
    activation checkpointing (see :class:`AttentionKeep`)."""
    return RopeAttentionFn.apply(qkv, cos, sin, seq_len, hq, hkv, d, keep, gen, rotated)


# QKV projection with RoPE in the GEMM epilogue (csrc/kernels/gemm_w4.hip, gemm_qkv_rope_w4): the
# hand-written 4-wave GEMM writes qkv with Q/K already rotated, so neither the separate RoPE
# kernel nor the rotated [T, (Hq + Hkv) D] copy exists; the flash kernels read Q/K from qkv.
# Default on (8B step: 1.001-1.003x, the RoPE forward kernel and the rotated copy gone; the
# kernel alone runs the Llama-3-8B QKV shape at 1.10-1.14x hipBLASLt, profiles/r3_gemm_w4_investigation.md);
# FT_QKV_ROPE=0 restores hipBLASLt + the RoPE kernel.
_QKV_ROPE = os.environ.get("FT_QKV_ROPE", "1") != "0"
_QKV_ROPE_MIN_K = 2048  # model dim from which the fused projection wins (see _qkv_rope_ok)


def set_qkv_rope(on: bool) -> None:
    global _QKV_ROPE
    _QKV_ROPE = bool(on)


def _qkv_rope_ok(x2: torch.Tensor, w: torch.Tensor, d: int) -> bool:
    if not (_QKV_ROPE and _W4_FWD and _GEMM_MODE != "blas" and x2.is_cuda and x2.dtype in _W4_DTYPES
            and w.dtype == x2.dtype):
        return False
    # K >= 2048 (the 8B-class projections): at GPT-2 sizes (K = 768 / 1024) the epilogue kernel
    # loses ~1 % of the step to hipBLASLt + the RoPE kernel (profiles/r3_gpt2_w4_ab.log)
    return d % 8 == 0 and x2.shape[1] >= _QKV_ROPE_MIN_K and _w4_fits(x2, w)


class QKVRopeFn(torch.autograd.Function):
    """qkv = x W^T with Q/K rotated (reference model.py:195 then :100-126). Backward receives the
    gradient of the unrotated projection (the attention backward already rotated dQ/dK back,
    :class:`RopeAttentionFn`), then dW / dX."""

    @staticmethod
    def forward(ctx, x2, w, sink, cos, sin, seq_len, hq, hkv, d):
        ctx.sink = sink
        ctx.cfg = (seq_len, hq, hkv, d)
        ctx.save_for_backward(x2, w, cos, sin)
        return kernels().gemm_qkv_rope_w4(x2, w, cos, sin, seq_len, hq, hkv, d)

    @staticmethod
    def backward(ctx, dq):
        x2, w, cos, sin = ctx.saved_tensors
        seq_len, hq, hkv, d = ctx.cfg
        dq = dq.contiguous()
        dw = weight_grad_async(dq, x2, ctx.sink)
        dx = mm_dx(dq, w)
        return dx, dw, None, None, None, None, None, None, None


def qkv_rope_attention(xn, wqkv, sink, cos, sin, seq_len, hq, hkv, d, keep: Optional[AttentionKeep] = None,
                       gen: int = -1):
    """QKV projection + RoPE + causal GQA attention (reference model.py:179-212). Returns o [.., Hq D]."""
    x2 = xn.reshape(-1, xn.shape[-1])
    if _qkv_rope_ok(x2, wqkv, d):
        qkv = QKVRopeFn.apply(x2.contiguous(), wqkv, sink, cos, sin, seq_len, hq, hkv, d)
        return rope_attention(qkv, cos, sin, seq_len, hq, hkv, d, keep, gen, rotated=True)
    qkv = linear(xn, wqkv, sink)
    return rope_attention(qkv.view(-1, qkv.shape[-1]), cos, sin, seq_len, hq, hkv, d, keep, gen)


# --------------------------------------------------------------------------------------
# SwiGLU on the fused [w1; w3] projection
# --------------------------------------------------------------------------------------
def swiglu_reference(gu: torch.Tensor) -> torch.Tensor:
    g, u = gu.chunk(2, dim=-1)
    return F.silu(g) * u


class SwiGLUFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, gu):
        ctx.save_for_backward(gu)
        if native(gu):
            return kernels().swiglu_fwd(gu.contiguous())
        return swiglu_reference(gu)

    @staticmethod
    def backward(ctx, da):
        (gu,) = ctx.saved_tensors
        if native(da):
            return kernels().swiglu_bwd(da.contiguous(), gu.contiguous())
        with torch.enable_grad():
            x = gu.detach().requires_grad_(True)
            (dx,) = torch.autograd.grad(swiglu_reference(x), (x,), da)
        return dx


def swiglu(gu):
    return SwiGLUFn.apply(gu)


_FUSED_FFN = os.environ.get("FT_FUSED_FFN", "1") != "0"
# FT_FFN_T_ONLY=1: the SwiGLU kernels write only the transposed activation / gradient and
# the w2 forward and w13 dX GEMMs read those transposed (A^T operand), saving one
# [T, F] and one [T, 2F] bf16 write per layer.
_FFN_T_ONLY = os.environ.get("FT_FFN_T_ONLY", "0") == "1"


def set_ffn_t_only(on: bool) -> None:
    global _FFN_T_ONLY
    _FFN_T_ONLY = bool(on)


# w1|w3 projection with SwiGLU in the GEMM epilogue (csrc/kernels/gemm_w4.hip, gemm_swiglu_w4): each
# 224-column tile holds g and u of the same 112 features, the epilogue writes gu (for the backward),
# a = silu(g) u and a^T, so the separate SwiGLU forward pass (a re-read of the [T, 2F] gu) is gone.
# 8B step 1.002x best / 1.003x median with a^T by in-register transposes (the first form, a^T
# gathered by 2-byte LDS reads, was 0.994x): profiles/r3_w4_swiglu_ab.log. FT_W4_SWIGLU=0: GEMM + swiglu_fwd_t.
_W4_SWIGLU = os.environ.get("FT_W4_SWIGLU", "1") != "0"


def set_w4_swiglu(on: bool) -> None:
    global _W4_SWIGLU
    _W4_SWIGLU = bool(on)


def _swiglu_w4_ok(x2: torch.Tensor, w13: torch.Tensor) -> bool:
    """Fused path: bf16 on the GPU, w4 tile shapes (T % 256, F % 112, K % 128), at least half the
    chip in tiles, and the transposed-operand weight-gradient path (which consumes a^T)."""
    if not (_W4_SWIGLU and _W4_FWD and _GEMM_MODE != "blas" and x2.is_cuda and x2.dtype == torch.bfloat16
            and w13.dtype == x2.dtype and not _FFN_T_ONLY):
        return False
    T, K = x2.shape
    F = w13.shape[0] // 2
    if T % 256 or K % 128 or F % 112 or (T // 256) * (F // 112) < _W4_MIN_TILES:
        return False
    return _DW_MODE == "all" or (_DW_MODE != "none" and 2.0 * T * 2 * F * K >= _DW_MIN_FLOP)


def _ffn_w4t_ok(x2: torch.Tensor, w13: torch.Tensor, w2: torch.Tensor) -> bool:
    """Every FFN product on the w4 kernel with no transposed operand anywhere: forward w1|w3 with the
    SwiGLU epilogue (F % 112), backward da on k-major w2 with the SwiGLU-backward epilogue, dW2 /
    dW13 on k-major dY and activations, dX on k-major w13 (bf16 or fp16)."""
    if not (_W4_SWIGLU and _W4_FWD and _W4_BWD and x2.is_cuda and x2.dtype in _W4_DTYPES
            and w13.dtype == x2.dtype and w2.dtype == x2.dtype):
        return False
    T, D = x2.shape
    F = w2.shape[1]
    if T % 256 or D % 128 or F % 112 or (T // 256) * (F // 112) < _W4_MIN_TILES:
        return False
    return (_w4t_fits(T, F, D, x2, w2) and _w4t_fits(2 * F, D, T, x2) and _w4t_fits(D, F, T, x2)
            and _w4t_fits(T, D, 2 * F, x2))


class FeedForwardW4Fn(torch.autograd.Function):
    """x -> [w1; w3] GEMM + SwiGLU -> w2 GEMM, every product on the w4 kernel, no transposes:

    forward   (gu, a) = gemm_swiglu_w4(x, w13)     SwiGLU in the epilogue, gu kept for backward
              y = a w2^T
    backward  dW2 = dy^T a                          k-major dy and a, sums of squares in the epilogue
              dgu = gemm_swiglu_bwd_w4(dy, w2, gu)  da = dy w2 (k-major w2), SwiGLU backward in the
                                                    epilogue: neither da nor a SwiGLU pass exists
              dW13 = dgu^T x ; dx = dgu w13         k-major dgu / x / w13
    Reference math: model.py:253-254."""

    @staticmethod
    def forward(ctx, x, w13, w2, sink13, sink2):
        K_ = kernels()
        D = x.shape[-1]
        x2 = x.reshape(-1, D).contiguous()
        gu, a, _ = K_.gemm_swiglu_w4(x2, w13, False)
        y = mm_fwd(a, w2)
        ctx.sinks = (sink13, sink2)
        ctx.xshape = x.shape
        ctx.save_for_backward(x2, gu, a, w13, w2)
        return y.view(*x.shape[:-1], w2.shape[0])

    @staticmethod
    def backward(ctx, dy):
        x2, gu, a, w13, w2 = ctx.saved_tensors
        sink13, sink2 = ctx.sinks
        dy2 = dy.reshape(-1, w2.shape[0]).contiguous()
        dw2 = weight_grad_async(dy2, a, sink2)
        dgu = kernels().gemm_swiglu_bwd_w4(dy2, w2, gu, 0)
        dw13 = weight_grad_async(dgu, x2, sink13)
        dx = mm_dx(dgu, w13).view(ctx.xshape)
        return dx, dw13, dw2, None, None


class FeedForwardFn(torch.autograd.Function):
    """x → [w1; w3] GEMM → SwiGLU → w2 GEMM as one autograd node (GPU, 64-multiple shapes).

    The tiled SwiGLU kernels also emit the transposed activation ``a^T`` (forward) and
    ``dgu^T`` (backward), the K-contiguous operands of the w2 and w13 weight-gradient GEMMs,
    so neither needs a separate transpose pass; only ``a^T`` is kept for backward (``a``
    itself is freed right after the w2 GEMM). Reference math: model.py:253-254."""

    @staticmethod
    def forward(ctx, x, w13, w2, sink13, sink2):
        K_ = kernels()
        D = x.shape[-1]
        x2 = x.reshape(-1, D)
        if _swiglu_w4_ok(x2, w13):
            gu, a, aT = K_.gemm_swiglu_w4(x2.contiguous(), w13)
            tn, t_only = True, False
        else:
            gu = mm_fwd(x2, w13)
            tn = _use_tn(gu, x2)
            t_only = tn and _FFN_T_ONLY
            if tn:
                a, aT = K_.swiglu_fwd_t(gu, not t_only)
            else:
                a, aT = K_.swiglu_fwd(gu), None
        y = torch.mm(aT.t(), w2.t()) if t_only else mm_fwd(a, w2)
        ctx.sinks = (sink13, sink2)
        ctx.tn = tn
        ctx.t_only = t_only
        ctx.xshape = x.shape
        ctx.save_for_backward(x2, gu, aT if tn else a, w13, w2)
        return y.view(*x.shape[:-1], w2.shape[0])

    @staticmethod
    def backward(ctx, dy):
        x2, gu, a_or_T, w13, w2 = ctx.saved_tensors
        sink13, sink2 = ctx.sinks
        K_ = kernels()
        dy2 = dy.reshape(-1, w2.shape[0]).contiguous()
        if ctx.tn:
            dw2 = weight_grad_async(dy2, None, sink2, xT=a_or_T)
        else:
            dw2 = weight_grad_async(dy2, a_or_T, sink2)
        da = torch.mm(dy2, w2)
        if ctx.tn:
            dgu, dguT = K_.swiglu_bwd_t(da, gu, not ctx.t_only)
            if ctx.t_only:
                dgu = dguT.t()
        else:
            dgu, dguT = K_.swiglu_bwd(da, gu), None
        del da
        dw13 = weight_grad_async(dgu, x2, sink13, dyT=dguT)
        dx = torch.mm(dgu, w13).view(ctx.xshape)
        return dx, dw13, dw2, None, None


class FusedFFNFn(torch.autograd.Function):
    """FFN on the hand GEMM with SwiGLU in the GEMM epilogues (csrc/kernels/gemm.hip):

    forward   (a, gu) = gemm_swiglu(x, w13)      a = silu(g) * u, gu = [g | u] kept for backward
              y = a @ w2^T
    backward  dW2 = dy^T a                       (row-major operands, no transpose)
              dgu = gemm_swiglu_bwd(dy, w2, gu)  da = dy @ w2 and the SwiGLU backward in one kernel
              dW13 = dgu^T x ; dx = dgu @ w13
    No separate activation kernel and no transposed copies. Reference math: model.py:253-254."""

    @staticmethod
    def forward(ctx, x, w13, w2, sink13, sink2):
        K_ = kernels()
        D = x.shape[-1]
        x2 = x.reshape(-1, D).contiguous()
        a, gu = K_.gemm_swiglu(x2, w13)
        y = mm_fwd(a, w2)
        ctx.sinks = (sink13, sink2)
        ctx.xshape = x.shape
        ctx.save_for_backward(x2, gu, a, w13, w2)
        return y.view(*x.shape[:-1], w2.shape[0])

    @staticmethod
    def backward(ctx, dy):
        x2, gu, a, w13, w2 = ctx.saved_tensors
        sink13, sink2 = ctx.sinks
        dy2 = dy.reshape(-1, w2.shape[0]).contiguous()
        dw2 = weight_grad_async(dy2, a, sink2)
        dgu = kernels().gemm_swiglu_bwd(dy2, w2, gu)
        dw13 = weight_grad_async(dgu, x2, sink13)
        dx = mm_dx(dgu, w13).view(ctx.xshape)
        return dx, dw13, dw2, None, None


def feed_forward(x, w13, w2, sink13=None, sink2=None):
    """SwiGLU FFN on the fused [w1; w3] weight; fused node on the GPU, composed ops on CPU."""
    if native(x) and _FUSED_FFN:
        T, D = x.numel() // x.shape[-1], x.shape[-1]
        F = w13.shape[0] // 2
        if _ffn_w4t_ok(x.reshape(T, D), w13, w2):
            return FeedForwardW4Fn.apply(x, w13, w2, sink13, sink2)
        # gemm_swiglu / gemm_swiglu_bwd tile T and F by 256 (BM / BN of the 256 kernel)
        if _hand("ffn", T, 2 * F, D, x, w13, w2) and F % 256 == 0 and T % 256 == 0:
            return FusedFFNFn.apply(x, w13, w2, sink13, sink2)
        if w13.shape[0] % 128 == 0 and T % 64 == 0:
            return FeedForwardFn.apply(x, w13, w2, sink13, sink2)
    return linear(swiglu(linear(x, w13, sink13)), w2, sink2)


# --------------------------------------------------------------------------------------
# LM head + cross-entropy (sum over tokens × 1/num_items)
# --------------------------------------------------------------------------------------
# Token rows per LM-head chunk: the [rows, V] bf16 logits of one chunk stay under this many MiB.
# Default 1 GiB: with V = 131072, seq 2048 (512 MiB of logits) runs as one chunk and seq 65536
# in 16 chunks of 4096 rows instead of a 16 GiB [T, V] logits tensor plus its gradient. On a
# 288 GB MI355X the half-GiB at seq 2048 is cheaper to keep than to split: two 256 MiB chunks
# measured 109.7 vs 107.5 ms/step (profiles/r2_head_chunk_ab.log) — the dX GEMM at M = 1024
# fills the chip worse and dW is accumulated twice.
_HEAD_CHUNK_MB = float(os.environ.get("FT_HEAD_CHUNK_MB", "1024"))


def _head_rows(T: int, V: int) -> int:
    rows = int(_HEAD_CHUNK_MB * 2**20) // (2 * V)
    rows = max(256, rows // 256 * 256)
    return min(T, rows)


# The head's dW from a chunk of dlogits: hipBLASLt on the row-major operands (no transposed
# copy of the 256 MiB chunk, which would double the chunk's footprint); FT_HEAD_DW_TN=1 uses
# the transposed ("TN") layout instead.
_HEAD_DW_TN = os.environ.get("FT_HEAD_DW_TN", "0") == "1"


def _dx_into(out: torch.Tensor, dy2: torch.Tensor, w: torch.Tensor) -> None:
    """out[T, K] = dy2[T, N] @ w[N, K]."""
    T, N = dy2.shape
    K = w.shape[1]
    if _w4_dx_ok(T, K, N, dy2, w) and out.is_contiguous():
        kernels().gemm_w4_ex(dy2, False, w, True, T, K, N, out, False, None, 0)
        return
    if _hand("dx", T, K, N, dy2, w):
        kernels().gemm(dy2, True, w, False, T, K, N, out, None, False, 0)
    else:
        torch.mm(dy2, w, out=out)


def _dw_into(out: torch.Tensor, dy2: torch.Tensor, x2: torch.Tensor, accumulate: bool,
             sink: Optional[GradSink] = None) -> None:
    """out[N, K] (+)= dy2[T, N]^T @ x2[T, K]. ``sink``: the final write of the sink's gradient
    (its norm partials come from this product's epilogue)."""
    T, N = dy2.shape
    K = x2.shape[1]
    if _w4t_fits(N, K, T, dy2, x2) and dy2.is_contiguous() and x2.is_contiguous():
        part = sink.part if sink is not None else None
        kernels().gemm_w4_ex(dy2, True, x2, True, N, K, T, out, accumulate, part, 0)
        if part is not None:
            sink.sq_done = True
        return
    if _hand("dw", N, K, T, dy2, x2):
        kernels().gemm(dy2, False, x2, False, N, K, T, out, None, accumulate, 0)
        return
    if _HEAD_DW_TN and _use_tn(dy2, x2):
        K_ = kernels()
        a, b = K_.transpose2d(dy2, None), K_.transpose2d(x2, None)
        if accumulate:
            out.addmm_(a, b.t())
        else:
            torch.mm(a, b.t(), out=out)
        return
    if accumulate:
        out.addmm_(dy2.t(), x2)
    else:
        torch.mm(dy2.t(), x2, out=out)


# The head's logits GEMM (h W^T, [T, V]) on the w4 kernel's 256-wide tiles as well (FT_W4_HEAD=0:
# hipBLASLt). The other forward products use the w4 kernel only up to tile width 6
# (FT_W4_FWD_MAX_NJ); the head takes the widest tile.
_W4_HEAD = os.environ.get("FT_W4_HEAD", "1") != "0"


def set_w4_head(on: bool) -> None:
    global _W4_HEAD
    _W4_HEAD = bool(on)


_W4_HEAD_MIN_K = 2048  # model dim from which the head's logits go to w4 (GPT-2 sizes: hipBLASLt)


def _head_fwd(h2: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    if _W4_HEAD and _W4_FWD and h2.shape[1] >= _W4_HEAD_MIN_K and _w4_fits(h2, w) and h2.is_contiguous():
        return kernels().gemm_nt_w4(h2, w, None, None, 0)
    return mm_fwd(h2, w)


class LMHeadCrossEntropyFn(torch.autograd.Function):
    """LM head + cross-entropy, chunked over token rows, gradients formed in the forward pass.

    Reference: logits = h @ W^T (model.py:379), then CE over the fp32 copy of the full
    [T, V] logits (train.py:101-102). Here, per chunk of rows (``_head_rows``): logits_c
    = h_c W^T (bf16), per-row log-sum-exp + NLL (xent_fwd), dlogits written in place
    (xent_bwd_, scaled by 1/num_items), then dh_c = dlogits_c W and dW (+)= dlogits_c^T h_c
    straight into the flat gradient buffer; the chunk's logits are freed before the next.
    Backward only applies the upstream gradient (a no-op kernel when it is 1, which it is
    for ``loss.backward()``) and marks the weight gradient ready. Under gradient
    accumulation (the sink already holds earlier micro-batches) the forward keeps only the
    per-row lse and backward recomputes each chunk's logits with the upstream gradient.
    """

    @staticmethod
    def forward(ctx, h, weight, sink, labels, inv_count):
        D = h.shape[-1]
        h2 = h.reshape(-1, D)
        lab = labels.reshape(-1)
        ctx.sink = sink
        ctx.hshape = h.shape
        ctx.native = native(h)  # (backward's g is the fp32 loss gradient whatever the model dtype)
        if not ctx.native:
            logits = torch.mm(h2, weight.t())
            loss = F.cross_entropy(logits.float(), lab, reduction="sum", ignore_index=IGNORE_INDEX) * inv_count
            ctx.save_for_backward(h2, weight, lab, inv_count)
            return loss
        K_ = kernels()
        h2 = h2.contiguous()
        lab = lab.contiguous()
        T, V = h2.shape[0], weight.shape[0]
        rows = _head_rows(T, V)
        need = ctx.needs_input_grad[0] or ctx.needs_input_grad[1] or sink is not None
        fused = need and not (sink is not None and sink.accumulate)
        ctx.fused = fused
        ctx.rows = rows
        inv = inv_count.float().reshape(1).contiguous()
        one = torch.ones(1, dtype=torch.float32, device=h.device)
        dh = torch.empty_like(h2) if fused else None
        dw = None
        if fused:
            dw = sink.buf.view(V, D) if sink is not None else torch.empty_like(weight)
        losses, lses = [], []
        for c, r0 in enumerate(range(0, T, rows)):
            hc, lc = h2[r0 : r0 + rows], lab[r0 : r0 + rows]
            logits = _head_fwd(hc, weight)
            lr, lse = K_.xent_fwd(logits, lc, IGNORE_INDEX)
            losses.append(lr)
            if fused:
                K_.xent_bwd_(logits, lc, lse, one, inv, IGNORE_INDEX)  # logits := dlogits
                _dx_into(dh[r0 : r0 + rows], logits, weight)
                _dw_into(dw, logits, hc, c > 0, sink if r0 + rows >= T else None)
            else:
                lses.append(lse)
            del logits
        loss = (losses[0] if len(losses) == 1 else torch.cat(losses)).sum() * inv_count
        if fused:
            ctx.save_for_backward(dh, dw if sink is None else None)
        else:
            ctx.save_for_backward(h2, weight, lab, inv, torch.cat(lses))
        return loss

    @staticmethod
    def backward(ctx, g):
        sink = ctx.sink
        if not ctx.native:
            h2, w, lab, inv_count = ctx.saved_tensors
            with torch.enable_grad():
                hr = h2.detach().requires_grad_(True)
                wr = w.detach().requires_grad_(True)
                logits = torch.mm(hr, wr.t())
                loss = F.cross_entropy(logits.float(), lab, reduction="sum", ignore_index=IGNORE_INDEX) * inv_count
                dh, dw = torch.autograd.grad(loss, (hr, wr), g)
            return dh.view(ctx.hshape), _write_weight_grad(sink, dw), None, None, None
        K_ = kernels()
        gf = g.detach().float().reshape(1).contiguous()
        if ctx.fused:
            dh, dw = ctx.saved_tensors
            K_.scale_by_(dh, gf)
            if sink is not None:
                K_.scale_by_(sink.buf, gf)
                if sink.sq_done:  # the epilogue's sums of squares were of the unscaled dW
                    sink.part.mul_(gf * gf)
                sink.ready()
                return dh.view(ctx.hshape), None, None, None, None
            K_.scale_by_(dw, gf)
            return dh.view(ctx.hshape), dw, None, None, None
        h2, w, lab, inv, lse = ctx.saved_tensors
        T, D = h2.shape
        V = w.shape[0]
        rows = ctx.rows
        dh = torch.empty_like(h2)
        dw = sink.buf.view(V, D) if sink is not None else torch.empty_like(w)
        acc0 = sink.accumulate if sink is not None else False
        for c, r0 in enumerate(range(0, T, rows)):
            hc, lc = h2[r0 : r0 + rows], lab[r0 : r0 + rows]
            logits = _head_fwd(hc, w)
            K_.xent_bwd_(logits, lc, lse[r0 : r0 + rows].contiguous(), gf, inv, IGNORE_INDEX)
            _dx_into(dh[r0 : r0 + rows], logits, w)
            _dw_into(dw, logits, hc, acc0 or c > 0, sink if r0 + rows >= T else None)
            del logits
        if sink is not None:
            sink.ready()
            return dh.view(ctx.hshape), None, None, None, None
        return dh.view(ctx.hshape), dw, None, None, None


def lm_head_cross_entropy(h, weight, labels, inv_count, sink=None):
    return LMHeadCrossEntropyFn.apply(h, weight, sink, labels, inv_count)
