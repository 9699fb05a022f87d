"""The Llama-3-8B backward GEMMs on the w4 kernel's k-major layouts vs hipBLASLt.

For each product of the step's backward (T = 2048, D = 4096, F = 14336, V = 131072):
  w4        gemm_w4_ex on the operands as stored (dX: k-major W; dW: k-major dY and X)
  blas_rm   torch.mm on the same row-major operands (what hipBLASLt gets without copies)
  blas_tn   torch.mm on pre-transposed K-contiguous copies (the round-3 path; the transpose
            kernels themselves are not timed here)
Kernel time from CUDA events over 20 back-to-back launches after 5 warm-ups.

    python scripts/gemm_w4t_bench.py
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
    return s.elapsed_time(e) / n * 1e3  # us


def main():
    K_ = kernels()
    T, D, F, V = 2048, 4096, 14336, 131072
    dev = "cuda"
    r = lambda *s: (torch.rand(*s, device=dev) * 2 - 1).bfloat16()
    # (name, kind, M, N, K): dX = dY[T, N_out] @ W[N_out, K_in]; dW = dY^T X
    prods = [
        ("qkv dX", "dx", T, D, 6144), ("wo dX", "dx", T, D, D), ("w13 dX", "dx", T, D, 2 * F),
        ("w2 dX (da)", "dx", T, F, D), ("head dX", "dx", T, D, V),
        ("qkv dW", "dw", 6144, D, T), ("wo dW", "dw", D, D, T), ("w13 dW", "dw", 2 * F, D, T),
        ("w2 dW", "dw", D, F, T), ("head dW", "dw", V, D, T),
    ]
    print(f"{'product':14s} {'M':>6s} {'N':>6s} {'K':>6s} | {'w4 us':>8s} {'TF/s':>6s} | {'blas_rm':>8s} "
          f"{'TF/s':>6s} | {'blas_tn':>8s} {'TF/s':>6s} | w4/rm  w4/tn", flush=True)
    for name, kind, M, N, Kd in prods:
        fl = 2.0 * M * N * Kd
        if kind == "dx":
            a = r(M, Kd)           # dY [T, N_out]
            b = r(Kd, N)           # W [N_out, K_in] as stored
            w4 = lambda: K_.gemm_w4_ex(a, False, b, True, M, N, Kd, None, False, None, 0)
            rm = lambda: torch.mm(a, b)
            bt = b.t().contiguous()
            tn = lambda: torch.mm(a, bt.t())
        else:
            a = r(Kd, M)           # dY [T, N_out] (A^T as stored)
            b = r(Kd, N)           # X [T, K_in]
            out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
            part = torch.empty((M // 256) * (N // 128), device=dev)
            w4 = lambda: K_.gemm_w4_ex(a, True, b, True, M, N, Kd, out, False, part, 0)
            rm = lambda: torch.mm(a.t(), b, out=out)
            at_, bt_ = a.t().contiguous(), b.t().contiguous()
            tn = lambda: torch.mm(at_, bt_.t(), out=out)
        t_w4, t_rm, t_tn = timeit(w4), timeit(rm), timeit(tn)
        tf = lambda t: fl / t / 1e6
        print(f"{name:14s} {M:6d} {N:6d} {Kd:6d} | {t_w4:8.1f} {tf(t_w4):6.0f} | {t_rm:8.1f} {tf(t_rm):6.0f} | "
              f"{t_tn:8.1f} {tf(t_tn):6.0f} | {t_rm / t_w4:5.2f} {t_tn / t_w4:5.2f}", flush=True)
        del a, b
        torch.cuda.empty_cache()
    # the fused w2 dX + SwiGLU backward vs hipBLASLt da + the element-wise SwiGLU backward
    dy, w2, gu = r(T, D), r(D, F), r(T, 2 * F)
    t_f = timeit(lambda: K_.gemm_swiglu_bwd_w4(dy, w2, gu, 0))
    t_u = timeit(lambda: K_.swiglu_bwd(torch.mm(dy, w2), gu))
    print(f"swiglu bwd fused {t_f:8.1f} us vs hipBLASLt + swiglu_bwd {t_u:8.1f} us ({t_u / t_f:.2f}x)", flush=True)


if __name__ == "__main__":
    main()
