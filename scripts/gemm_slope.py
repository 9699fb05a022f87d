"""Per-K-tile cost of the 128-tile hand GEMM vs hipBLASLt: time vs K at fixed output shapes
(graph-timed, as scripts/gemm_small_bench.py), plus the 1-tile floor."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from fault_tolerant_llm_training_amd._native import kernels

K_ = kernels()


def graph_time(fn, it=20):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(it):
            fn()
    best = 1e30
    for _ in range(5):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        g.replay()
        b.record()
        torch.cuda.synchronize()
        best = min(best, a.elapsed_time(b) / it * 1e3)
    return best


def r(*shape):
    return (torch.rand(*shape, device="cuda") * 2 - 1).bfloat16()


for M, N in ((128, 128), (2048, 768), (2048, 2048), (4096, 4096)):
    for Kd in (64, 256, 1024, 4096):
        a, b = r(M, Kd), r(N, Kd)
        line = f"[{M:5d}x{N:5d}x{Kd:5d}] tiles128 {M * N // 16384:4d}"
        K_.gemm_config(128)
        h = graph_time(lambda: K_.gemm(a, True, b, True, M, N, Kd, None, None, False, 1))
        line += f"  hand128 {h:7.1f}"
        K_.gemm_config(0)
        bl = graph_time(lambda: torch.mm(a, b.t()))
        print(line + f"  blas {bl:7.1f} us", flush=True)
