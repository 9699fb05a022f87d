"""128x128-tile hand GEMM vs the 256-tile kernel vs hipBLASLt on the
GPT-2-small / -medium step shapes (T = 2048), MI355X.

Each variant is timed as 20 calls captured in one HIP graph (no host launch cost in the
number: these kernels run 5-40 us, about the host's launch time). Checks every variant
against fp32 torch.mm first.
    python scripts/gemm_small_bench.py [--llama]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch

from fault_tolerant_llm_training_amd._native import kernels

T = 2048
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
    g.replay()
    torch.cuda.synchronize()
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


cases = []
for tag, d, f, qkv, L in (("s", 768, 2048, 2304, 12), ("m", 1024, 2816, 3072, 24)):
    cases += [(f"{tag} fwd qkv", "nt", T, qkv, d, L), (f"{tag} fwd wo", "nt", T, d, d, L),
              (f"{tag} fwd w13", "nt", T, 2 * f, d, L), (f"{tag} fwd w2", "nt", T, d, f, L),
              (f"{tag} dX qkv", "nn", T, d, qkv, L), (f"{tag} dX wo", "nn", T, d, d, L),
              (f"{tag} dX w13", "nn", T, d, 2 * f, L), (f"{tag} dX w2", "nn", T, f, d, L),
              (f"{tag} dW qkv", "tn", qkv, d, T, L), (f"{tag} dW wo", "tn", d, d, T, L),
              (f"{tag} dW w13", "tn", 2 * f, d, T, L), (f"{tag} dW w2", "tn", d, f, T, L)]
if "--llama" in sys.argv:
    cases = [("8b fwd qkv", "nt", T, 6144, 4096, 32), ("8b dX wo", "nn", T, 4096, 4096, 32),
             ("8b dW wo", "tn", 4096, 4096, T, 32)]

variants = [("h128", 128), ("h256", 256)]
tot = {v[0]: 0.0 for v in variants}
tot["blas"] = tot["best"] = 0.0
for name, kind, M, N, Kd, cnt in cases:
    fl = 2.0 * M * N * Kd
    if kind == "nt":
        a, b = r(M, Kd), r(N, Kd)
        hand = lambda: K_.gemm(a, True, b, True, M, N, Kd, None, None, False, 0)
        blas = lambda: torch.mm(a, b.t())
        ref = a.float() @ b.float().t()
    elif kind == "nn":
        a, b = r(M, Kd), r(Kd, N)
        hand = lambda: K_.gemm(a, True, b, False, M, N, Kd, None, None, False, 0)
        blas = lambda: torch.mm(a, b)
        ref = a.float() @ b.float()
    else:
        a, b = r(Kd, M), r(Kd, N)
        hand = lambda: K_.gemm(a, False, b, False, M, N, Kd, None, None, False, 0)
        blas = lambda: torch.mm(a.t(), b)
        ref = a.float().t() @ b.float()
    line = f"{name:10s} [{M:5d}x{N:5d}x{Kd:5d}]"
    best = 1e30
    for vn, tile in variants:
        if tile == 256 and (M % 256 or N % 256):
            line += f" | {vn} {'-':>6s}"
            continue
        K_.gemm_config(tile)
        out = hand()
        err = ((out.float() - ref).norm() / ref.norm()).item()
        assert err < 1e-2, (name, vn, err)
        t = graph_time(hand)
        tot[vn] += t * cnt / 1e3
        best = min(best, t)
        line += f" | {vn} {t:6.1f}"
    K_.gemm_config(0)
    tb = graph_time(blas)
    tot["blas"] += tb * cnt / 1e3
    tot["best"] += min(best, tb) * cnt / 1e3
    line += f" | blas {tb:6.1f} us ({fl / tb / 1e6:4.0f} TF) | best hand x{tb / best:4.2f} ({fl / best / 1e6:4.0f} TF)"
    print(line, flush=True)
print("per-step totals (ms): " + ", ".join(f"{k} {v:.2f}" for k, v in tot.items()))
