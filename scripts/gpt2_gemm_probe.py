"""GPT-2-sized products (T = 2048 tokens) on the w4 kernel with a forced tile width / split-K vs
hipBLASLt (torch.mm): which of the products the host plan leaves on hipBLASLt could run in-tree.

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
             ("qkv dX", "dx", T, D, W), ("wo dX", "dx", T, D, D), ("w13 dX", "dx", T, D, 2 * F),
             ("qkv dW", "dw", W, D, T), ("wo dW", "dw", D, D, T), ("w13 dW", "dw", 2 * F, D, T),
             ("w2 dW", "dw", D, F, T)]
    for name, lay, M, N, Kd in prods:
        if lay == "fwd":
            a, b = r(M, Kd), r(N, Kd)
            blas = lambda: torch.mm(a, b.t())  # noqa: E731
            w4 = lambda nj, sp: K_.gemm_nt_w4(a, b, None, None, nj, sp)  # noqa: E731
        elif lay == "dx":
            a, b = r(M, Kd), r(Kd, N)
            blas = lambda: torch.mm(a, b)  # noqa: E731
            w4 = lambda nj, sp: K_.gemm_w4_ex(a, False, b, True, M, N, Kd, None, False, None, nj, sp)  # noqa: E731
        else:  # dW = dY^T X, both operands k-major as stored (no split-K on this layout)
            a, b = r(Kd, M), r(Kd, N)
            blas = lambda: torch.mm(a.t(), b)  # noqa: E731
            w4 = lambda nj, sp: K_.gemm_w4_ex(a, True, b, True, M, N, Kd, None, False, None, nj, sp)  # noqa: E731
        tb = timeit(blas)
        cells = []
        if M % 256:
            print(f"{name:8s} {M}x{N}x{Kd}: hipBLASLt {tb:6.1f} us | M % 256 != 0: no w4 tile", flush=True)
            continue
        for nj in (4, 6, 8):
            if N % (32 * nj):
                continue
            tiles = (M // 256) * (N // (32 * nj))
            for sp in ((1,) if lay == "dw" else (1, 2, 3, 4, 6, 8)):
                if Kd // 128 < sp or tiles * sp > 512:
                    continue
                cells.append((timeit(lambda: w4(nj, sp)), nj, sp, tiles * sp))
        best = min(cells)
        print(f"{name:8s} {M}x{N}x{Kd}: hipBLASLt {tb:6.1f} us | w4 best {best[0]:6.1f} us (nj {best[1]} x{best[2]}, "
              f"{best[3]} WGs) = {tb / best[0]:.2f}x | " + " ".join(f"{nj}x{sp}:{t:.1f}" for t, nj, sp, _ in cells),
              flush=True)


if __name__ == "__main__":
    main()
