"""Per-tile fixed cost of the w4 GEMM by layout: time vs K at a fixed output grid (one round of
256 tiles of 256 x 256, and four rounds), with and without the epilogue's global stores
(gemm_w4_set_dbg(1)). t(K) = a + b K: b is the main loop's cost per K-tile, a the tile's fixed
cost (launch, pipeline fill, epilogue); the store-ablated intercept shows the epilogue stores' share.

    python scripts/w4_overhead_probe.py
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


def fit(xs, ys):
    n = len(xs)
    mx, my = sum(xs) / n, sum(ys) / n
    b = sum((x - mx) * (y - my) for x, y in zip(xs, ys)) / sum((x - mx) ** 2 for x in xs)
    return my - b * mx, b


def main():
    K_ = kernels()
    r = lambda *s: (torch.rand(*s, device="cuda") * 2 - 1).bfloat16()  # noqa: E731
    Ks = [512, 1024, 2048, 4096, 8192]
    for M, N in ((4096, 4096), (8192, 8192)):
        rounds = (M // 256) * (N // 256) // 256
        for layout in ("fwd", "dx", "dw"):
            for dbg in (0, 1):
                K_.gemm_w4_set_dbg(dbg)
                ts = []
                for Kd in Ks:
                    if layout == "fwd":
                        a, b = r(M, Kd), r(N, Kd)
                        fn = lambda: K_.gemm_nt_w4(a, b, None, None, 8, 1)  # noqa: E731
                    elif layout == "dx":
                        a, b = r(M, Kd), r(Kd, N)
                        fn = lambda: K_.gemm_w4_ex(a, False, b, True, M, N, Kd, None, False, None, 8, 1)  # noqa: E731
                    else:
                        a, b = r(Kd, M), r(Kd, N)
                        fn = lambda: K_.gemm_w4_ex(a, True, b, True, M, N, Kd, None, False, None, 8, 1)  # noqa: E731
                    ts.append(timeit(fn))
                    del a, b
                ia, sl = fit([k / 64 for k in Ks], ts)
                cells = "  ".join(f"K{k}:{t:7.1f}" for k, t in zip(Ks, ts))
                print(f"{M}x{N} ({rounds} rounds) {layout:3s} stores={'off' if dbg else 'on '} | per round: "
                      f"fixed {ia / rounds:6.2f} us + {sl / rounds * 1e3:6.1f} ns/K-tile "
                      f"({2 * 256 * 256 * 64 * 256 / (sl / rounds * 1e-6) / 1e12:6.0f} TF/s loop) | {cells}", flush=True)
    K_.gemm_w4_set_dbg(0)


if __name__ == "__main__":
    main()
