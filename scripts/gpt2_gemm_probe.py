"""GPT-2-sized products (T = 2048 tokens) on the w4 kernel vs hipBLASLt (torch.mm): the automatic
plan (tile width, split-K), every forced plan, and the layouts as the step runs them -- forward
x W^T, dX = dY W (k-major W), dW = dY^T X (k-major dY and X, split-K since round 6, tail tile for
V % 256) -- including the LM head at V = 50304 / 131072.

    python scripts/gpt2_gemm_probe.py [dim ffn qkv_width]     (default GPT-2-small: 768 2048 2304)
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fault_tolerant_llm_training_amd._native import kernels  # noqa: E402


def timeit(fn, n=20, w=5):
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
    D, F, W = (int(v) for v in sys.argv[1:4]) if len(sys.argv) >= 4 else (768, 2048, 2304)
    T = 2048
    r = lambda *s: (torch.rand(*s, device="cuda") * 2 - 1).bfloat16()  # noqa: E731
    # (name, layout, M, N, K)
    prods = [("wo fwd", "fwd", T, D, D), ("w2 fwd", "fwd", T, D, F), ("w13 fwd", "fwd", T, 2 * F, D),
             ("qkv fwd", "fwd", T, W, D), ("head50k fwd", "fwd", T, 50304, D), ("head131k fwd", "fwd", T, 131072, D),
             ("qkv dX", "dx", T, D, W), ("wo dX", "dx", T, D, D), ("w13 dX", "dx", T, D, 2 * F),
             ("w2 dX", "dx", T, F, D), ("head50k dX", "dx", T, D, 50304),
             ("qkv dW", "dw", W, D, T), ("wo dW", "dw", D, D, T), ("w13 dW", "dw", 2 * F, D, T),
             ("w2 dW", "dw", D, F, T), ("head50k dW", "dw", 50304, D, T), ("head131k dW", "dw", 131072, D, T)]
    for name, lay, M, N, Kd in prods:
        if lay == "fwd":
            a, b = r(M, Kd), r(N, Kd)
            blas = lambda: torch.mm(a, b.t())  # noqa: E731
            w4 = lambda nj, sp: K_.gemm_nt_w4(a, b, None, None, nj, sp)  # noqa: E731
        elif lay == "dx":
            a, b = r(M, Kd), r(Kd, N)
            blas = lambda: torch.mm(a, b)  # noqa: E731
            w4 = lambda nj, sp: K_.gemm_w4_ex(a, False, b, True, M, N, Kd, None, False, None, nj, sp)  # noqa: E731
        else:  # dW = dY^T X, both operands k-major as stored
            a, b = r(Kd, M), r(Kd, N)
            blas = lambda: torch.mm(a.t(), b)  # noqa: E731
            w4 = lambda nj, sp: K_.gemm_w4_ex(a, True, b, True, M, N, Kd, None, False, None, nj, sp)  # noqa: E731
        tb = timeit(blas)
        auto = list(K_.gemm_w4_plan(M, N, Kd, lay == "dw", lay != "fwd"))
        ta = timeit(lambda: w4(0, 0)) if auto[0] else float("nan")
        cells = []
        big = M * N > 2048 * 40000
        for nj in (4, 6, 8):
            if N % (32 * nj):
                continue
            tiles = ((M + 255) // 256) * (N // (32 * nj))
            for sp in ((1,) if big else (1, 2, 3, 4, 6, 8)):
                if Kd // 128 < sp or (tiles * sp > 512 and sp > 1) or (lay == "dw" and sp > 1 and nj != 4):
                    continue
                cells.append((timeit(lambda: w4(nj, sp)), nj, sp, tiles * sp))
        best = min(cells)
        print(f"{name:13s} {M}x{N}x{Kd}: hipBLASLt {tb:7.1f} us | w4 auto {auto[0]}x{auto[1]} {ta:7.1f} us = "
              f"{tb / ta:.2f}x | best {best[0]:7.1f} us (nj {best[1]} x{best[2]}, {best[3]} WGs) = {tb / best[0]:.2f}x | "
              + " ".join(f"{nj}x{sp}:{t:.1f}" for t, nj, sp, _ in cells), flush=True)


if __name__ == "__main__":
    main()
