"""GEMM routing table (docs / tests): the kernel every GEMM of a step takes, from the same
predicates the autograd functions in ops/functional.py and ops/attention.py evaluate, for a preset
and dtype, on shape / dtype specs (nothing is allocated; no GPU needed). tests/test_routing_cpu.py
pins it per preset.
"""
from . import attention as A
from . import functional as Fx


class _Spec:
    """The routing-relevant attributes of a tensor (shape, dtype, device) without storage."""

    def __init__(self, *shape, dtype, cuda=True):
        self.shape, self.dtype, self.is_cuda = tuple(shape), dtype, cuda

    def is_contiguous(self):
        return True


def _w4_name(M, N, K, a_t, b_t):
    nj, sp = Fx._w4_plan(M, N, K, a_t, b_t)
    return f"w4 {32 * nj}" + (f" x{sp}" if sp > 1 else "")


def routing_table(margs, dtype, tokens: int = 2048, cuda: bool = True) -> dict:
    """{product: kernel} for one transformer layer and the LM head of ``margs`` at ``tokens`` rows:
    "w4 <tile width>[ xS]" (S = K slices), "w4 qkv+rope", "w4 swiglu", "w4 swiglu-bwd", "gemm_s",
    "f32 mfma" (fp32 models: csrc/kernels/gemm_f32.hip), or "hipBLASLt"."""
    T, D, V = tokens, margs.dim, margs.vocab_size
    hd, Hq, Hkv, Fh = margs.head_dim, margs.n_heads, margs.kv_heads, margs.ffn_hidden
    W = (Hq + 2 * Hkv) * hd
    sp = lambda *s: _Spec(*s, dtype=dtype, cuda=cuda)  # noqa: E731
    x, wqkv, wo, w13, w2, head = sp(T, D), sp(W, D), sp(D, Hq * hd), sp(2 * Fh, D), sp(D, Fh), sp(V, D)

    def fwd(xx, w):
        Tn, K = xx.shape
        N = w.shape[0]
        if Fx._s_ok(xx, w):
            return "gemm_s"
        if Fx._w4_fwd_ok(Tn, N, K, xx, w):
            return _w4_name(Tn, N, K, False, False)
        return "f32 mfma" if Fx.f32_route(Tn, N, K, False, False, xx, w) else "hipBLASLt"

    def dx(Tn, K, N, w):
        if Fx._w4_dx_ok(Tn, K, N, sp(Tn, N), w):
            return _w4_name(Tn, K, N, False, True)
        return "f32 mfma" if Fx.f32_route(Tn, K, N, False, True, sp(Tn, N), w) else "hipBLASLt"

    def dw(Tn, N, K):
        if Fx._w4_dw_ok(Tn, N, K, sp(Tn, N), sp(Tn, K)):
            return _w4_name(N, K, Tn, True, True)
        return "f32 mfma" if Fx._f32_dw_ok(Tn, N, K, sp(Tn, N), sp(Tn, K)) else "hipBLASLt"

    t = {}
    t["qkv fwd"] = "w4 qkv+rope" if A._qkv_rope_ok(x, wqkv, hd) else fwd(x, wqkv)
    t["qkv dX"], t["qkv dW"] = dx(T, D, W, wqkv), dw(T, W, D)
    t["wo fwd"], t["wo dX"], t["wo dW"] = fwd(sp(T, Hq * hd), wo), dx(T, Hq * hd, D, wo), dw(T, D, Hq * hd)
    if cuda and Fx._ffn_w4t_ok(x, w13, w2):
        t["w13 fwd"], t["w2 dX"] = "w4 swiglu", "w4 swiglu-bwd"
    else:
        t["w13 fwd"], t["w2 dX"] = fwd(x, w13), dx(T, Fh, D, w2)
    t["w13 dX"], t["w13 dW"] = dx(T, D, 2 * Fh, w13), dw(T, 2 * Fh, D)
    t["w2 fwd"], t["w2 dW"] = fwd(sp(T, Fh), w2), dw(T, D, Fh)
    rows = Fx._head_rows(T, V)
    t["head fwd"], t["head dX"], t["head dW"] = fwd(sp(rows, D), head), dx(rows, D, V, head), dw(rows, V, D)
    return t
