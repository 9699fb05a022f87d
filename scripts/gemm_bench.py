"""Hand-written gfx950 GEMM vs hipBLASLt (torch.mm) at every Llama-3-8B step shape, MI355X.

Each product is timed in the layout the step reads it in (forward NT, dX NN, dW TN on the
row-major activations, i.e. no transposes for the hand kernel), on uniform random data,
interleaved in one process. Prints us, TF/s, max relative error vs fp32.
    python scripts/gemm_bench.py [--quick]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch

from fault_tolerant_llm_training_amd._native import kernels

T = 2048
D, F, V, L = 4096, 14336, 131072, 32
QKV = 6144


def timeit(fn, it=10):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it * 1e3


def r(*shape):
    return (torch.rand(*shape, device="cuda") * 2 - 1).bfloat16()


K_ = kernels()
quick = "--quick" in sys.argv
cases = [
    ("fwd qkv", "nt", T, QKV, D, L), ("fwd wo", "nt", T, D, D, L), ("fwd w13", "nt", T, 2 * F, D, L),
    ("fwd w2", "nt", T, D, F, L), ("fwd head", "nt", T, V, D, 1),
    ("dX qkv", "nn", T, D, QKV, L), ("dX wo", "nn", T, D, D, L), ("dX w13", "nn", T, D, 2 * F, L),
    ("dX w2", "nn", T, F, D, L), ("dX head", "nn", T, D, V, 1),
    ("dW qkv", "tn", QKV, D, T, L), ("dW wo", "tn", D, D, T, L), ("dW w13", "tn", 2 * F, D, T, L),
    ("dW w2", "tn", D, F, T, L), ("dW head", "tn", V, D, T, 1),
]
if quick:
    cases = [c for c in cases if c[0] in ("fwd w13", "dX w13", "dW w13", "fwd head")]
if "--gpt2" in sys.argv:  # GPT-2-small / -medium (d 768 / 1024) at seq 2048, V = 131072
    cases = []
    for tag, d, f, qkv, L in (("s", 768, 2048, 2304, 12), ("m", 1024, 2816, 3072, 24)):
        cases += [(f"{tag} fwd qkv", "nt", T, qkv, d, L), (f"{tag} fwd wo", "nt", T, d, d, L),
                  (f"{tag} fwd w13", "nt", T, 2 * f, d, L), (f"{tag} fwd w2", "nt", T, d, f, L),
                  (f"{tag} fwd head", "nt", T, V, d, 1), (f"{tag} dX qkv", "nn", T, d, qkv, L),
                  (f"{tag} dX wo", "nn", T, d, d, L), (f"{tag} dX w13", "nn", T, d, 2 * f, L),
                  (f"{tag} dX w2", "nn", T, f, d, L), (f"{tag} dX head", "nn", T, d, V, 1),
                  (f"{tag} dW qkv", "tn", qkv, d, T, L), (f"{tag} dW w13", "tn", 2 * f, d, T, L),
                  (f"{tag} dW head", "tn", V, d, T, 1)]
tot_h = tot_b = 0.0
for name, kind, M, N, Kd, cnt in cases:
    fl = 2.0 * M * N * Kd
    if kind == "nt":   # y = x @ W^T: x [M, K], W [N, K]
        a, b = r(M, Kd), r(N, Kd)
        hand = lambda: K_.gemm(a, True, b, True, M, N, Kd, None, None, False, 0)
        blas = lambda: torch.mm(a, b.t())
        ref = lambda: a.float() @ b.float().t()
    elif kind == "nn":  # dx = dy @ W: dy [M, K], W [K, N]
        a, b = r(M, Kd), r(Kd, N)
        hand = lambda: K_.gemm(a, True, b, False, M, N, Kd, None, None, False, 0)
        blas = lambda: torch.mm(a, b)
        ref = lambda: a.float() @ b.float()
    else:               # dW = dy^T @ x: dy [K=T, M], x [K=T, N]
        a, b = r(Kd, M), r(Kd, N)
        hand = lambda: K_.gemm(a, False, b, False, M, N, Kd, None, None, False, 0)
        blas = lambda: torch.mm(a.t(), b)
        ref = lambda: a.float().t() @ b.float()
    out = hand()
    rf = ref()
    err = ((out.float() - rf).norm() / rf.norm()).item()
    del rf
    th, tb = timeit(hand), timeit(blas)
    tot_h += th * cnt / 1e3
    tot_b += tb * cnt / 1e3
    print(f"{name:9s} [{M:6d}x{N:6d}x{Kd:6d}] hand {th:8.1f} us {fl / th / 1e6:6.0f} TF | hipBLASLt {tb:8.1f} us "
          f"{fl / tb / 1e6:6.0f} TF | x{tb / th:4.2f} | relerr {err:.1e}", flush=True)
print(f"per-step GEMM total: hand {tot_h:.2f} ms, hipBLASLt {tot_b:.2f} ms")
