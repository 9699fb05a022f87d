"""w4 GEMM plans (tile width x split-K) vs hipBLASLt on the Llama-3-8B dX / forward products.

For each product: the automatic plan, every forced (nj, splits) that fits, and hipBLASLt on the
row-major operands and on K-contiguous ("TN") copies (copies not timed). Kernel time from CUDA
events over back-to-back launches after warm-ups, uniform random bf16 in [-1, 1).

    python scripts/w4_split_bench.py [--only dx|fwd]
"""
import argparse
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
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default="")
    a = ap.parse_args()
    K_ = kernels()
    T, D, F, V = 2048, 4096, 14336, 131072
    r = lambda *s: (torch.rand(*s, device="cuda") * 2 - 1).bfloat16()  # noqa: E731
    prods = [("qkv dX", "dx", T, D, 6144), ("wo dX", "dx", T, D, D), ("w13 dX", "dx", T, D, 2 * F),
             ("head dX", "dx", T, D, V), ("wo fwd", "fwd", T, D, D), ("w2 fwd", "fwd", T, D, F),
             ("qkv fwd", "fwd", T, 6144, D)]
    for name, kind, M, N, Kd in prods:
        if a.only and kind != a.only:
            continue
        fl = 2.0 * M * N * Kd
        tf = lambda t: fl / t / 1e6  # noqa: E731
        x = r(M, Kd)
        if kind == "dx":
            w = r(Kd, N)
            run = lambda nj, sp: K_.gemm_w4_ex(x, False, w, True, M, N, Kd, None, False, None, nj, sp)  # noqa: E731
            wt = w.t().contiguous()
            blas_rm, blas_tn = (lambda: torch.mm(x, w)), (lambda: torch.mm(x, wt.t()))
            auto = tuple(K_.gemm_w4_plan(M, N, Kd, False, True))
        else:
            w = r(N, Kd)
            run = lambda nj, sp: K_.gemm_nt_w4(x, w, None, None, nj, sp)  # noqa: E731
            blas_rm = blas_tn = lambda: torch.mm(x, w.t())
            auto = tuple(K_.gemm_w4_plan(M, N, Kd, False, False))
        res = []
        for nj in (8, 7, 6, 4):
            if N % (32 * nj):
                continue
            for sp in (1, 2):
                if sp == 2 and Kd % 256:
                    continue
                t = timeit(lambda: run(nj, sp))
                res.append((t, nj, sp))
        t_rm, t_tn = timeit(blas_rm), timeit(blas_tn)
        best = min(res)
        ta = next(t for t, nj, sp in res if (nj, sp) == auto)
        cells = "  ".join(f"{nj}x{sp}:{t:7.1f}" for t, nj, sp in res)
        print(f"{name:8s} {M}x{N}x{Kd} | auto {auto[0]}x{auto[1]} {ta:7.1f} us {tf(ta):5.0f} TF/s | best "
              f"{best[1]}x{best[2]} {best[0]:7.1f} | blas rm {t_rm:7.1f} tn {t_tn:7.1f} ({tf(t_tn):5.0f}) | "
              f"tn/auto {t_tn / ta:5.2f} | {cells}", flush=True)
        del x, w
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
