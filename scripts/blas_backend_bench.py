"""hipBLASLt vs rocBLAS (ATen's two bf16 GEMM backends on ROCm) at every Llama-3-8B step product.

Each product in the layout the step issues it (forward x W^T, dX dY W, dW via the transposed
"TN" operands), random bf16 data, interleaved in one process.
    python scripts/blas_backend_bench.py
"""
import torch

T, D, F, V, QKV = 2048, 4096, 14336, 131072, 6144


def timeit(fn, it=10):
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


cases = [("fwd qkv", T, QKV, D), ("fwd wo", T, D, D), ("fwd w13", T, 2 * F, D), ("fwd w2", T, D, F),
         ("fwd head", T, V, D), ("dX qkv", T, D, QKV), ("dX wo", T, D, D), ("dX w13", T, D, 2 * F),
         ("dX w2", T, F, D), ("dX head", T, D, V), ("dW qkv", QKV, D, T), ("dW wo", D, D, T),
         ("dW w13", 2 * F, D, T), ("dW w2", D, F, T), ("dW head", V, D, T)]
for name, M, N, K in cases:
    if name.startswith("fwd"):
        a, b = r(M, K), r(N, K)
        fn = lambda: torch.mm(a, b.t())
    elif name.startswith("dX"):
        a, b = r(M, K), r(K, N)
        fn = lambda: torch.mm(a, b)
    else:  # TN on transposed copies: a = dY^T [M, T], b = X^T [N, T]
        a, b = r(M, K), r(N, K)
        fn = lambda: torch.mm(a, b.t())
    fl = 2.0 * M * N * K
    res = {}
    for lib in ("cublaslt", "cublas", "cublaslt", "cublas"):
        torch.backends.cuda.preferred_blas_library(lib)
        res.setdefault(lib, []).append(timeit(fn))
    tl, tr = min(res["cublaslt"]), min(res["cublas"])
    print(f"{name:9s} [{M:6d}x{N:6d}x{K:6d}] hipBLASLt {tl:7.1f} us {fl / tl / 1e6:5.0f} TF | rocBLAS {tr:7.1f} us "
          f"{fl / tr / 1e6:5.0f} TF | rocBLAS/hipBLASLt speed x{tl / tr:4.2f}", flush=True)
torch.backends.cuda.preferred_blas_library("cublaslt")
