"""fp32 GEMM: the hand-written MFMA kernel (gemm_f32) vs hipBLASLt (torch.mm on the same stored
operands, as the fp32 model path called it before) on the products of an fp32 GPT-2-small /
-medium / Llama-3-8B layer at T = 2048 tokens. Event-timed, median of 20 after 5 warm-up calls.

    python scripts/gemm_f32_bench.py [--dma 0|1]
"""
import os
import sys

import torch

sys.path.insert(0, os.getcwd())
from fault_tolerant_llm_training_amd._native import kernels  # noqa: E402


def timeit(f, reps=20, warm=5):
    for _ in range(warm):
        f()
    ts = []
    for _ in range(reps):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        f()
        e.record()
        e.synchronize()
        ts.append(s.elapsed_time(e) * 1e3)
    ts.sort()
    return ts[len(ts) // 2]


def main():
    K_ = kernels()
    if len(sys.argv) > 2 and sys.argv[1] == "--dma":  # A/B: LDS-DMA form (1, default) or registers (0)
        K_.gemm_f32_set_dma(int(sys.argv[2]))
    T = 2048
    cfgs = {"gpt2-small": (768, 2048, 50304), "gpt2-medium": (1024, 2816, 50304), "llama3-8b": (4096, 14336, 131072)}
    print(f"{'product':28s} {'M':>6} {'N':>6} {'K':>6} | {'f32 mfma us':>11} {'TF/s':>6} | {'hipBLASLt us':>12} {'TF/s':>6} | ratio")
    for name, (D, F, V) in cfgs.items():
        prods = [("qkv fwd", T, 3 * D, D, "fwd"), ("w13 fwd", T, 2 * F, D, "fwd"), ("w2 fwd", T, D, F, "fwd"),
                 ("w13 dX", T, D, 2 * F, "dx"), ("w2 dX", T, F, D, "dx"), ("w13 dW", 2 * F, D, T, "dw"),
                 ("w2 dW", D, F, T, "dw"), ("head fwd", T, V if D < 4096 else V // 4, D, "fwd")]
        for pn, M, N, Kd, kind in prods:
            r = lambda *s: torch.rand(*s, device="cuda") * 2 - 1  # noqa: E731
            if kind == "fwd":  # x [M, K] @ w[N, K]^T
                a, b = r(M, Kd), r(N, Kd)
                f1 = lambda: K_.gemm_f32(a, False, b, False, M, N, Kd)  # noqa: E731
                f0 = lambda: torch.mm(a, b.t())  # noqa: E731
            elif kind == "dx":  # dy [M, K] @ w [K, N]
                a, b = r(M, Kd), r(Kd, N)
                f1 = lambda: K_.gemm_f32(a, False, b, True, M, N, Kd)  # noqa: E731
                f0 = lambda: torch.mm(a, b)  # noqa: E731
            else:  # dy [K, M]^T @ x [K, N]
                a, b = r(Kd, M), r(Kd, N)
                f1 = lambda: K_.gemm_f32(a, True, b, True, M, N, Kd)  # noqa: E731
                f0 = lambda: torch.mm(a.t(), b)  # noqa: E731
            t1, t0 = timeit(f1), timeit(f0)
            fl = 2.0 * M * N * Kd
            print(f"{name + ' ' + pn:28s} {M:6d} {N:6d} {Kd:6d} | {t1:11.1f} {fl / t1 / 1e6:6.1f} | {t0:12.1f} "
                  f"{fl / t0 / 1e6:6.1f} | {t0 / t1:5.2f}", flush=True)
            del a, b


if __name__ == "__main__":
    main()
