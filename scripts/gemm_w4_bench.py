"""w4 GEMM (csrc/kernels/gemm_w4.hip) vs hipBLASLt (torch.mm), forward (NT) layout, Llama-3-8B step
shapes, every tile width that divides N (nj: BN = 32 nj) and the automatic pick; correctness vs fp32
first. Interleaved rounds, one process, uniform random [-1, 1) bf16 (cdna_hip_programming.md §5.4
rules 24-25).   python scripts/gemm_w4_bench.py [--rounds R]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from fault_tolerant_llm_training_amd._native import kernels

K_ = kernels()


def r(*s):
    return (torch.rand(*s, device="cuda") * 2 - 1).bfloat16()


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


for M, N, K in [(256, 256, 64), (2048, 6144, 4096), (768, 1792, 640)]:
    a, b = r(M, K), r(N, K)
    ref = a.float() @ b.float().t()
    for nj in (8, 7, 6, 4):
        if N % (32 * nj):
            continue
        err = ((K_.gemm_nt_w4(a, b, None, None, nj).float() - ref).norm() / ref.norm()).item()
        print(f"check {M}x{N}x{K} nj={nj}: rel {err:.2e} {'OK' if err < 4e-3 else 'FAIL'}", flush=True)
        if err >= 4e-3:
            sys.exit(1)
rounds = int(sys.argv[sys.argv.index("--rounds") + 1]) if "--rounds" in sys.argv else 3
T, D, F, V = 2048, 4096, 14336, 131072
shapes = [("qkv", T, 6144, D), ("wo", T, D, D), ("w13", T, 2 * F, D), ("w2", T, D, F), ("head", T, V, D),
          # weight gradients dW[N_out, K_in] = dY^T X on the transposed operands (NT, K = tokens)
          ("dWqkv", 6144, D, T), ("dWwo", D, D, T), ("dWw13", 2 * F, D, T), ("dWw2", D, F, T), ("dWhead", V, D, T)]
res = {}
for rd in range(rounds):
    for name, M, N, K in shapes:
        a, b = r(M, K), r(N, K)
        o = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        fns = {f"nj{nj}": (lambda nj=nj: K_.gemm_nt_w4(a, b, o, None, nj)) for nj in (8, 7, 6, 4) if N % (32 * nj) == 0}
        fns["blas"] = lambda: torch.mm(a, b.t(), out=o)
        for k, fn in fns.items():
            res.setdefault((name, k), []).append(timeit(fn, 10 if name == "head" else 20))
for name, M, N, K in shapes:
    fl = 2.0 * M * N * K
    keys = [k for (n_, k) in res if n_ == name]
    med = {k: sorted(res[(name, k)])[len(res[(name, k)]) // 2] for k in keys}
    pick = f"nj{K_.gemm_w4_pick(M, N)}"
    print(f"{name:5s} [{M:6d}x{N:6d}x{K:6d}] " + " | ".join(f"{k} {med[k]:7.1f} us {fl / med[k] / 1e6:5.0f} TF"
                                                      for k in keys)
          + f" | pick {pick}: x{med['blas'] / med[pick]:.3f} of blas", flush=True)
