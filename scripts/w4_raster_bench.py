"""Grouped tile raster of the w4 GEMM (gemm_w4_set_group) on the Llama-3-8B products, routed as
in the step (tile width and split-K from the host plan). Each XCD runs 32 tiles at a time from a
contiguous range of the raster; group = G sweeps bands of G slow-dimension tiles, so those 32 tiles
form a G x 32/G block (fewer distinct operand panels per K-step in the XCD's L2) instead of a
1-2-row strip (group 0). The groups alternate three times per product; best of the three.

    python scripts/w4_raster_bench.py [groups...]     (default 0 2 4 8)
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fault_tolerant_llm_training_amd._native import kernels  # noqa: E402


def timeit(fn, n=10, w=3):
    for _ in range(w):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n * 1e3


def main():
    K_ = kernels()
    groups = [int(g) for g in sys.argv[1:]] or [0, 2, 4, 8]
    T, D, F, V = 2048, 4096, 14336, 131072
    r = lambda *s: (torch.rand(*s, device="cuda") * 2 - 1).bfloat16()  # noqa: E731
    prods = [
        ("wo fwd", "fwd", T, D, D), ("w2 fwd", "fwd", T, D, F), ("head fwd", "fwd", T, V, D),
        ("w13 fwd swiglu", "swiglu", T, 2 * F, D),
        ("qkv dX", "dx", T, D, 6144), ("wo dX", "dx", T, D, D), ("w13 dX", "dx", T, D, 2 * F),
        ("head dX", "dx", T, D, V), ("w2 dX swiglu-bwd", "swbwd", T, F, D),
        ("qkv dW", "dw", 6144, D, T), ("wo dW", "dw", D, D, T), ("w13 dW", "dw", 2 * F, D, T),
        ("w2 dW", "dw", D, F, T), ("head dW", "dw", V, D, T),
    ]
    print("product            " + "".join(f"   G={g:<4d}" for g in groups) + "  best/G0", flush=True)
    tot = {g: 0.0 for g in groups}
    for name, kind, M, N, Kd in prods:
        if kind == "fwd":
            a, b = r(M, Kd), r(N, Kd)
            fn = lambda: K_.gemm_nt_w4(a, b, None, None)  # noqa: E731
        elif kind == "swiglu":
            a, b = r(M, Kd), r(N, Kd)
            fn = lambda: K_.gemm_swiglu_w4(a, b, True)  # noqa: E731
        elif kind == "dx":
            a, b = r(M, Kd), r(Kd, N)
            fn = lambda: K_.gemm_w4_ex(a, False, b, True, M, N, Kd, None, False, None, 0)  # noqa: E731
        elif kind == "swbwd":
            a, b, gu = r(T, D), r(D, F), r(T, 2 * F)
            fn = lambda: K_.gemm_swiglu_bwd_w4(a, b, gu, 0)  # noqa: E731
        else:
            a, b = r(Kd, M), r(Kd, N)
            out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
            part = torch.empty((M // 256) * (N // 128), device="cuda")
            fn = lambda: K_.gemm_w4_ex(a, True, b, True, M, N, Kd, out, False, part, 0)  # noqa: E731
        best = {g: 1e30 for g in groups}
        for _ in range(3):
            for g in groups:
                K_.gemm_w4_set_group(g)
                best[g] = min(best[g], timeit(fn))
        K_.gemm_w4_set_group(-1)
        for g in groups:
            tot[g] += best[g]
        b0 = best[groups[0]]
        print(f"{name:18s} " + "".join(f" {best[g]:8.1f}" for g in groups) + f"  {b0 / min(best.values()):6.3f}",
              flush=True)
        del a, b, fn
        torch.cuda.empty_cache()
    print(f"{'sum':18s} " + "".join(f" {tot[g]:8.1f}" for g in groups), flush=True)


if __name__ == "__main__":
    main()
