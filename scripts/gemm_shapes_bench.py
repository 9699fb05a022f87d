"""Per-call GEMM timing of one Llama-3-8B training step (hipBLASLt via torch.mm), MI355X.

Every GEMM the step issues (ops/functional.py), at the exact operand layouts, with the
alternative layout of the same product (C^T = B^T A^T: hipBLASLt picks different tiles),
so the weak shapes show up. Prints us, TF/s and the per-step ms the call contributes.
"""
import torch

T = 2048
D, F, V, L = 4096, 14336, 131072, 32
QKV = 6144


def timeit(fn, it=20):
    for _ in range(3):
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


rows = []
total_ms = 0.0
total_alt = 0.0
# (name, M, N, K, per-step count): out[M, N] = A[M, K] @ B[N, K]^T  (fwd / dW TN) or A @ B[K, N] (dX)
cases = [
    ("fwd qkv", "nt", T, QKV, D, L), ("fwd wo", "nt", T, D, D, L), ("fwd w13", "nt", T, 2 * F, D, L),
    ("fwd w2", "nt", T, D, F, L), ("fwd head", "nt", T, V, D, 1),
    ("dX qkv", "nn", T, D, QKV, L), ("dX wo", "nn", T, D, D, L), ("dX w13", "nn", T, D, 2 * F, L),
    ("dX w2", "nn", T, F, D, L), ("dX head", "nn", T, D, V, 1),
    ("dW qkv", "tn", QKV, D, T, L), ("dW wo", "tn", D, D, T, L), ("dW w13", "tn", 2 * F, D, T, L),
    ("dW w2", "tn", D, F, T, L), ("dW head", "tn", V, D, T, 1),
]
for name, kind, M, N, K, cnt in cases:
    fl = 2.0 * M * N * K
    if kind == "nt":      # y[M,N] = x[M,K] @ W[N,K]^T
        a, b = r(M, K), r(N, K)
        out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        outT = torch.empty(N, M, device="cuda", dtype=torch.bfloat16)
        f = lambda: torch.mm(a, b.t(), out=out)
        g = lambda: torch.mm(b, a.t(), out=outT)  # y^T = W @ x^T
    elif kind == "nn":    # dx[M,N] = dy[M,K] @ W[K,N]
        a, b = r(M, K), r(K, N)
        out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        outT = torch.empty(N, M, device="cuda", dtype=torch.bfloat16)
        f = lambda: torch.mm(a, b, out=out)
        g = lambda: torch.mm(b.t(), a.t(), out=outT)
    else:                 # dW[M,N] = dyT[M,K] @ xT[N,K]^T (K = tokens contiguous)
        a, b = r(M, K), r(N, K)
        out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        outT = torch.empty(N, M, device="cuda", dtype=torch.bfloat16)
        f = lambda: torch.mm(a, b.t(), out=out)
        g = lambda: torch.mm(b, a.t(), out=outT)
    t0 = timeit(f)
    t1 = timeit(g)
    total_ms += t0 * cnt / 1e3
    total_alt += min(t0, t1) * cnt / 1e3
    print(f"{name:9s} [{M:6d}x{N:6d}x{K:6d}] {t0:8.1f} us {fl / t0 / 1e6:6.0f} TF | swapped {t1:8.1f} us "
          f"{fl / t1 / 1e6:6.0f} TF | x{cnt} = {t0 * cnt / 1e3:6.2f} ms/step", flush=True)
    del a, b, out, outT
print(f"GEMM total {total_ms:.2f} ms/step (best-of-two layouts {total_alt:.2f} ms/step)")
