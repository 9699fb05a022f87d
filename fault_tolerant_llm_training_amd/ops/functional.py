"""Autograd functions of the transformer hot path.

GPU tensors run the hand-written gfx950 kernels in ``csrc/kernels`` (loaded by
:func:`fault_tolerant_llm_training_amd._native.kernels`, which raises if the
library is missing). Every bf16 / fp16 GEMM of the Llama-3-8B and GPT-2 presets runs on the
hand-written w4 MFMA kernel (``csrc/kernels/gemm_w4.h``; the routing table per preset is pinned by
``tests/test_routing_cpu.py``); the fp32 models' GEMMs run on the hand-written fp32 MFMA kernel
(``csrc/kernels/gemm_f32.hip``, v_mfma_f32_16x16x4_f32); hipBLASLt (``torch.mm`` / ``torch.addmm``)
remains for fp64 models and for shapes no hand-written tile fits.
Model dtypes (``--model-dtype``): bf16 (every kernel), fp16 (every kernel; the MFMA GEMM and
flash kernels in their fp16 variants), fp32 (the element-wise / reduction kernels in fp32,
fp32 attention kernels, the fp32 MFMA GEMM).
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

# ---------------------------------------------------------------------------------------------
# GEMM routing. Every product of the step runs on the hand-written gfx950 "w4" kernel
# (csrc/kernels/gemm_w4.h) on its operands as stored -- forward x W^T (K-contiguous), dX = dY W
# (k-major W), dW = dY^T X (k-major dY and X, into the flat gradient buffer with the gradient-norm
# partials in the epilogue). The GPT-2-sized products (18-96 tiles at one sequence per GPU) take a
# deterministic K split (the dW layout too since round 6) and, for the LM-head dW at V = 50304, a
# tail tile (M % 256). Per-product plans and measurements: profiles/r6/gpt2_gemm_probe_*.log,
# profiles/r5_w4_split_bench.log; the routing table per preset: tests/test_routing_cpu.py.
# set_w4_small(False) (FT_W4_SMALL=0) restores the round-5 routing of the small products to
# hipBLASLt (A/B); the 128 x 128-tile kernel (gemm_s.hip, set_gemm_s) is opt-in.
# ---------------------------------------------------------------------------------------------
# FT_GEMM_BLAS=1: every GEMM on hipBLASLt (and the separate RoPE / SwiGLU kernels): the plain
# reference path of convergence comparisons (scripts/gpu_convergence.sh)
_BLAS_ONLY = os.environ.get("FT_GEMM_BLAS", "0") == "1"
_W4_FWD = True   # forward products on w4 (A/B: set_w4_fwd)
_W4_BWD = os.environ.get("FT_W4_BWD", "1") != "0"  # backward products on w4 (A/B: the hipBLASLt backward)
_W4_DTYPES = (torch.bfloat16, torch.float16)  # bf16 / fp16 MFMA variants of the kernel
# fp32 models: the fp32 MFMA kernel (gemm_f32.hip) for every product it takes (K % 32; a k-major
# operand with rows % 4); FT_F32_MFMA=0 / set_f32_mfma(False): hipBLASLt (A/B)
_F32_MFMA = os.environ.get("FT_F32_MFMA", "1") != "0"


def set_f32_mfma(on: bool) -> None:
    global _F32_MFMA
    _F32_MFMA = bool(on)


def f32_route(M: int, N: int, K: int, a_t: bool, b_t: bool, *ts) -> bool:
    """C[M, N] over K on the fp32 MFMA kernel? fp32 CUDA operands, K % 32, a k-major A with
    M % 4 / B with N % 4 (float4 rows), 16-B aligned rows."""
    if _BLAS_ONLY or not _F32_MFMA or not all(t.is_cuda and t.dtype == torch.float32 for t in ts):
        return False
    return K % 32 == 0 and K > 0 and (not a_t or M % 4 == 0) and (not b_t or N % 4 == 0) and all(
        t.shape[-1] % 4 == 0 for t in ts)
# Workgroups (output tiles x K slices) a product needs before it goes to the w4 kernel: half the
# chip. (Tests lower it to drive small shapes through the same paths.)
_W4_MIN_TILES = 128
_W4_SHORT_K = 1024
_W4_DEEP_K = 4096
_W4_SMALL = os.environ.get("FT_W4_SMALL", "1") != "0"  # round 6: the GPT-2-sized products on w4 too
_W4_SMALL_WGS = 16  # ... from this many workgroups (the GPT-2-small wo dW: 18 tiles x 3 slices)


def set_w4_small(on: bool) -> None:
    global _W4_SMALL
    _W4_SMALL = bool(on)


def set_w4_fwd(on: bool) -> None:
    global _W4_FWD
    _W4_FWD = bool(on)


def set_w4_bwd(on: bool) -> None:
    global _W4_BWD
    _W4_BWD = bool(on)


@functools.lru_cache(maxsize=512)
def _w4_plan(M: int, N: int, K: int, a_t: bool, b_t: bool):
    """(tile width / 32, K slices) of the w4 kernel's automatic plan for C[M, N] over K; (0, 1) when
    no tile width fits N."""
    return tuple(kernels().gemm_w4_plan(M, N, K, a_t, b_t))


def _w4_wgs(M: int, N: int, K: int, a_t: bool, b_t: bool) -> int:
    """Workgroups of the w4 kernel's automatic plan for C[M, N] over K (0: no plan)."""
    nj, sp = _w4_plan(M, N, K, a_t, b_t)
    return -(-M // 256) * (N // (32 * nj)) * sp if nj else 0


def set_w4_splitk(mode: int) -> None:
    """Split-K of the w4 kernel (FT_W4_SPLITK): 0 off, 1 automatic (default), 2 forced where it fits."""
    kernels().gemm_w4_set_splitk(int(mode))
    _w4_plan.cache_clear()


def w4_route(M: int, N: int, K: int, a_t: bool, b_t: bool, *ts) -> bool:
    """C[M, N] over a K-deep sum on the w4 kernel? 16-bit CUDA operands of one dtype, M % 256 (the
    dW layout: M % 8, a tail tile), K % 128, a tile width for N, and a plan of enough workgroups."""
    if _BLAS_ONLY or not (all(t.is_cuda and t.dtype in _W4_DTYPES for t in ts) and len({t.dtype for t in ts}) == 1):
        return False
    if (M % 256 and not (a_t and M % 8 == 0)) or K % 128 or K < 128:  # K-tiles of 64 in pairs
        return False
    nj, splits = _w4_plan(M, N, K, a_t, b_t)
    if nj == 0:
        return False
    wgs = -(-M // 256) * (N // (32 * nj)) * splits
    if _W4_SMALL:
        return wgs >= min(_W4_MIN_TILES, _W4_SMALL_WGS)
    if M % 256:
        return False
    if a_t:  # dW (round 5: never split)
        return wgs >= _W4_MIN_TILES
    # forward / dX below a full round (GPT-2 sizes, profiles/r5_gpt2_gemm_probe.log): short
    # reductions (K <= 1024: wo forward / dX on 48-64 tiles, 1.15-1.39x hipBLASLt) and deep
    # split ones (K >= 4096: w1|w3 dX, 1.14-1.25x) win; the 2048-3072-deep ones in between lose
    # (w2 forward 0.82-0.88x, -medium qkv dX 0.94x)
    return wgs >= 256 or (K <= _W4_SHORT_K and wgs >= 32) or (K >= _W4_DEEP_K and wgs >= _W4_MIN_TILES)


# GPT-2-sized forward products on the 128 x 128-tile kernel (csrc/kernels/gemm_s.hip): K <= 1024
# and at least 256 output tiles. Alone (graph-timed) it runs GPT-2-small qkv 1.20x / w13 1.10x,
# -medium qkv 1.05x / w13 1.15x hipBLASLt (profiles/r3_gemm_s_vs_hipblaslt.log), inside the
# graph-replayed step 0.99-1.00x (profiles/r3_gpt2_s_ab.log): opt-in (set_gemm_s).
_GEMM_S = False


def set_gemm_s(on: bool) -> None:
    global _GEMM_S
    _GEMM_S = bool(on)


def _s_ok(x2: torch.Tensor, w: torch.Tensor) -> bool:
    if not (_GEMM_S and not _BLAS_ONLY and x2.is_cuda and x2.dtype in _W4_DTYPES and w.dtype == x2.dtype):
        return False
    T, K = x2.shape
    N = w.shape[0]
    return T % 128 == 0 and N % 128 == 0 and K % 64 == 0 and K <= 1024 and (T // 128) * (N // 128) >= 256


# A forward product on the widest (256-column) w4 tile only from K = 2048: at GPT-2 sizes (K = 768 /
# 1024) the wide tile's prologue / epilogue outweigh its main loop (LM-head logits 439 vs 362 us
# for hipBLASLt at K = 768, profiles/r4_gpt2_head_fwd_probe.log); the narrower tiles run there.
_W4_WIDE_MIN_K = 2048


def _w4_fwd_ok(T: int, N: int, K: int, x2, w) -> bool:
    """The forward product on w4; before round 6 the 256-wide tile below K = 2048 only within one
    round (the GPT-2-medium w1|w3: 176 tiles, 27.7 vs 35.0 us for hipBLASLt). Since round 6
    (_W4_SMALL) the GPT-2 LM head at V = 131072, K = 768 / 1024 runs on it too: 0.79x hipBLASLt
    there, the 128-wide tile 0.60x (profiles/r6/gpt2_gemm_probe_small.log)."""
    if not (_W4_FWD and w.is_contiguous() and w4_route(T, N, K, False, False, x2, w)):
        return False
    nj, sp = _w4_plan(T, N, K, False, False)
    return _W4_SMALL or K >= _W4_WIDE_MIN_K or nj <= 6 or (T // 256) * (N // (32 * nj)) * sp <= 256


def mm_fwd(x2: torch.Tensor, w: torch.Tensor, residual: Optional[torch.Tensor] = None) -> torch.Tensor:
    """y = x2 @ w^T (+ residual, in the epilogue): x2 [T, K], w [N, K] (nn.Linear layout)."""
    T, K = x2.shape
    N = w.shape[0]
    res = None if residual is None else residual.reshape(T, N).contiguous()
    if _s_ok(x2, w):
        return kernels().gemm_nt_s(x2.contiguous(), w, None, res, 1)
    if _w4_fwd_ok(T, N, K, x2, w):
        return kernels().gemm_nt_w4(x2.contiguous(), w, None, res, 0, 0)
    if w.is_contiguous() and f32_route(T, N, K, False, False, x2, w):
        return kernels().gemm_f32(x2.contiguous(), False, w, False, T, N, K, None, False, None, res)
    if residual is None:
        return torch.mm(x2, w.t())
    return torch.addmm(residual.reshape(T, N), x2, w.t())


def _w4_dx_ok(T: int, K: int, N: int, dy2: torch.Tensor, w: torch.Tensor) -> bool:
    """dX[T, K] = dY[T, N] W[N, K] on w4 (k-major W read as stored). The deep reductions (the 8B
    w1|w3 dX, N = 2F; the LM-head dX, N = V) whose 256-wide tiles fill half the chip take a K split
    (profiles/r5_w4_split_bench.log)."""
    return _W4_BWD and w.is_contiguous() and w4_route(T, K, N, False, True, dy2, w)


def mm_dx(dy2: torch.Tensor, w: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """dx = dy2 @ w: dy2 [T, N], w [N, K]."""
    T, N = dy2.shape
    K = w.shape[1]
    if _w4_dx_ok(T, K, N, dy2, w) and (out is None or out.is_contiguous()):
        return kernels().gemm_w4_ex(dy2.contiguous(), False, w, True, T, K, N, out, False, None, 0, 0)
    if w.is_contiguous() and (out is None or out.is_contiguous()) and f32_route(T, K, N, False, True, dy2, w):
        return kernels().gemm_f32(dy2.contiguous(), False, w, True, T, K, N, out, False, None, None)
    if out is not None:
        return torch.mm(dy2, w, out=out)
    return torch.mm(dy2, w)


def _w4_dw_ok(T: int, N: int, K: int, dy2: torch.Tensor, x2: torch.Tensor) -> bool:
    return (_W4_BWD and dy2.is_contiguous() and x2.is_contiguous()
            and w4_route(N, K, T, True, True, dy2, x2))


def _f32_dw_ok(T: int, N: int, K: int, dy2: torch.Tensor, x2: torch.Tensor) -> bool:
    return dy2.is_contiguous() and x2.is_contiguous() and f32_route(N, K, T, True, True, dy2, x2)


def _f32_dw(dy2, x2, out, accumulate: bool, sink: Optional[GradSink]):
    """dW = dy2^T x2 on the fp32 MFMA kernel (k-major operands read as stored), (+)= into ``out``,
    with the sink's norm partials (of the stored values, as the w4 dW epilogue) when ``sink`` is
    given: the product that writes the sink's final gradient."""
    T, N = dy2.shape
    K = x2.shape[1]
    part = sink.part if sink is not None else None
    r = kernels().gemm_f32(dy2, True, x2, True, N, K, T, out, accumulate, part, None)
    if part is not None:
        sink.sq_done = True
    return r


def weight_grad(dy2: torch.Tensor, x2: torch.Tensor, sink: Optional[GradSink]):
    """dW[N, K] = dy2[T, N]^T @ x2[T, K], into the sink (flat grad buffer) or returned."""
    T, N = dy2.shape
    K = x2.shape[1]
    if _w4_dw_ok(T, N, K, dy2, x2):
        # both operands read as stored (k-major A and B), straight into the sink, with the norm
        # partials of the stored gradient from the epilogue
        if sink is None:
            return kernels().gemm_w4_ex(dy2, True, x2, True, N, K, T, None, False, None, 0, 0)
        kernels().gemm_w4_ex(dy2, True, x2, True, N, K, T, sink.buf.view(N, K), sink.accumulate, sink.part, 0, 0)
        if sink.part is not None:
            sink.sq_done = True
        sink.ready()
        return None
    if _f32_dw_ok(T, N, K, dy2, x2):
        if sink is None:
            return _f32_dw(dy2, x2, None, False, None)
        _f32_dw(dy2, x2, sink.buf.view(N, K), sink.accumulate, sink)
        sink.ready()
        return None
    if sink is not None:
        sink.mm(dy2.t(), x2)
        return None
    return torch.mm(dy2.t(), x2)


# Weight-gradient GEMMs that do not take the w4 kernel (hipBLASLt: the small presets) run on a side
# stream (set_dw_stream): dW and the dX GEMM of the same node are independent, and small products
# leave CUs idle when run one after the other (8B step on the round-1 routing: 108.6 -> 107.1 ms,
# profiles/r1_dw_stream_ab.log). The side stream waits for the compute stream before each dW (so
# it sees dY / X), and the bucket hooks fired from it order the reducer's collectives after it.
# join_dw_stream() (GradReducer.finish, FlatAdamW.step) makes the compute stream wait for every dW
# before the optimizer. The w4 dW GEMMs run inline (_W4_DW_SIDE): they hold one workgroup per CU,
# a concurrent dX kernel cannot co-reside, so the side stream only adds cross-stream waits (8B
# step 108.5 -> 106.9 ms with dW inline, profiles/r4_ab.log).
_DW_STREAM = True
_dw_streams = {}
_dw_pending = {}  # device -> FIFO of (dW done event, operands kept alive until then)
_DW_LAG = 4  # dW GEMMs the compute stream may run ahead by
_W4_DW_SIDE = False


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


def weight_grad_async(dy2: torch.Tensor, x2: torch.Tensor, sink: Optional[GradSink]):
    """:func:`weight_grad` into ``sink`` on the dW side stream (or inline)."""
    if not (_DW_STREAM and dy2.is_cuda and sink is not None):
        return weight_grad(dy2, x2, sink)
    dy2 = dy2.contiguous()
    x2 = x2.contiguous()
    T, N, K = dy2.shape[0], dy2.shape[1], x2.shape[1]
    if not _W4_DW_SIDE and _w4_dw_ok(T, N, K, dy2, x2) and _w4_wgs(N, K, T, True, True) >= 256:
        # a full-chip w4 dW runs inline; the GPT-2-sized ones (54-192 workgroups) run on the side
        # stream beside the dX product of the same node, which leaves the rest of the CUs idle too
        return weight_grad(dy2, x2, sink)
    # Operand lifetime is stream-ordered instead of record_stream(): the operands stay referenced in
    # a short FIFO; before one is dropped the compute stream waits for its dW, so the freed blocks
    # are reusable by the compute stream at once (record_stream() kept every recorded activation
    # out of the caching allocator until its event completed: HBM at ~1.6x the allocated peak,
    # profiles/r1_allocator_pools.log).
    cur = torch.cuda.current_stream(dy2.device)
    side = _dw_side(dy2.device)
    side.wait_stream(cur)
    with torch.cuda.stream(side):
        weight_grad(dy2, x2, sink)
        ev = torch.cuda.Event()
        ev.record()
    q = _dw_pending.setdefault(_dev_key(dy2.device), collections.deque())
    q.append((ev, (dy2, x2)))
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


# w1|w3 projection with SwiGLU in the GEMM epilogue (csrc/kernels/gemm_w4.h, gemm_swiglu_w4): each
# 224-column tile holds g and u of the same 112 features, the epilogue writes gu (for the backward)
# and a = silu(g) u, so the separate SwiGLU forward pass (a re-read of the [T, 2F] gu) is gone
# (8B step 1.002-1.003x, profiles/r3_w4_swiglu_ab.log; set_w4_swiglu(False): GEMM + SwiGLU kernels).
_W4_SWIGLU = True


def set_w4_swiglu(on: bool) -> None:
    global _W4_SWIGLU
    _W4_SWIGLU = bool(on)


def _ffn_w4t_ok(x2: torch.Tensor, w13: torch.Tensor, w2: torch.Tensor) -> bool:
    """Every FFN product on the w4 kernel with no transposed operand anywhere: forward w1|w3 with the
    SwiGLU epilogue (a tile width of 16 NJ features for F, no K split: gemm_swiglu_pick; the 8B F =
    14336 at 112 features, GPT-2 at 64 / 128), backward da on k-major w2 with the SwiGLU-backward
    epilogue, dW2 / dW13 on k-major dY and activations, dX on k-major w13 (bf16 or fp16)."""
    if not (_W4_SWIGLU and _W4_FWD and _W4_BWD and w13.is_contiguous() and w2.is_contiguous()):
        return False
    T, D = x2.shape
    F = w2.shape[1]
    if T % 256 or D % 128:
        return False
    nj = _swiglu_nj(T, F)
    if nj == 0 or (T // 256) * (F // (16 * nj)) < (min(_W4_MIN_TILES, _W4_SMALL_WGS) if _W4_SMALL else _W4_MIN_TILES):
        return False
    if not _W4_SMALL and F % 112:
        return False
    return (w4_route(T, F, D, False, True, x2, w2) and w4_route(2 * F, D, T, True, True, x2, w13)
            and w4_route(D, F, T, True, True, x2, w2) and w4_route(T, D, 2 * F, False, True, x2, w13))


@functools.lru_cache(maxsize=64)
def _swiglu_nj(T: int, F: int) -> int:
    return int(kernels().gemm_swiglu_pick(T, F))


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
    """x -> [w1; w3] GEMM -> SwiGLU kernel -> w2 GEMM as one autograd node (GPU shapes the w4 FFN
    does not take: the GPT-2-sized presets, fp32). Weight gradients go into the sinks; ``a`` is kept
    for dW2 and ``gu`` for the SwiGLU backward. Reference math: model.py:253-254."""

    @staticmethod
    def forward(ctx, x, w13, w2, sink13, sink2):
        K_ = kernels()
        D = x.shape[-1]
        x2 = x.reshape(-1, D)
        gu = mm_fwd(x2, w13)
        a = K_.swiglu_fwd(gu)
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
        dgu = kernels().swiglu_bwd(mm_dx(dy2, w2), gu)
        dw13 = weight_grad_async(dgu, x2, sink13)
        dx = mm_dx(dgu, w13).view(ctx.xshape)
        return dx, dw13, dw2, None, None


def feed_forward(x, w13, w2, sink13=None, sink2=None):
    """SwiGLU FFN on the fused [w1; w3] weight; fused node on the GPU, composed ops on CPU."""
    if native(x):
        T, D = x.numel() // x.shape[-1], x.shape[-1]
        if _ffn_w4t_ok(x.reshape(T, D), w13, w2):
            return FeedForwardW4Fn.apply(x, w13, w2, sink13, sink2)
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


def _dx_into(out: torch.Tensor, dy2: torch.Tensor, w: torch.Tensor) -> None:
    """out[T, K] = dy2[T, N] @ w[N, K]."""
    mm_dx(dy2, w, out)


def _dw_into(out: torch.Tensor, dy2: torch.Tensor, x2: torch.Tensor, accumulate: bool,
             sink: Optional[GradSink] = None) -> None:
    """out[N, K] (+)= dy2[T, N]^T @ x2[T, K]. ``sink``: the final write of the sink's gradient
    (its norm partials come from this product's epilogue)."""
    T, N = dy2.shape
    K = x2.shape[1]
    if _w4_dw_ok(T, N, K, dy2, x2):
        part = sink.part if sink is not None else None
        kernels().gemm_w4_ex(dy2, True, x2, True, N, K, T, out, accumulate, part, 0, 0)
        if part is not None:
            sink.sq_done = True
        return
    if _f32_dw_ok(T, N, K, dy2, x2) and out.is_contiguous():
        _f32_dw(dy2, x2, out, accumulate, sink)
        return
    if accumulate:
        out.addmm_(dy2.t(), x2)
    else:
        torch.mm(dy2.t(), x2, out=out)


def _head_fwd(h2: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    return mm_fwd(h2.contiguous(), w)


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


# attention ops live in ops/attention.py; re-exported for callers of the functional namespace
from .attention import (  # noqa: E402,F401
    AttentionKeep,
    QKVRopeFn,
    RopeAttentionFn,
    attention_reference,
    qkv_rope_attention,
    rope_attention,
    rope_reference,
    set_qkv_rope,
)
