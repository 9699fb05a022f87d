"""Micro-benchmark: weight-gradient GEMM layouts on MI355X (hipBLASLt via torch.mm).

dW[N, K] = dY^T[N, T] @ X[T, K]. Current call: mm(dY.t(), X) (both operands T-major, "NT").
Alternative: transposed copies so the reduction dim (T) is contiguous for both ("TN").
"""
import torch

T = 2048
shapes = {  # name: (N_out, K_in)
    "qkv": (6144, 4096), "wo": (4096, 4096), "w13": (28672, 4096), "w2": (4096, 14336), "head": (131072, 4096),
}


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
    return s.elapsed_time(e) / it * 1e3  # us


for name, (N, K) in shapes.items():
    dy = torch.randn(T, N, device="cuda").bfloat16()
    x = torch.randn(T, K, device="cuda").bfloat16()
    w = torch.randn(N, K, device="cuda").bfloat16()
    out = torch.empty(N, K, device="cuda", dtype=torch.bfloat16)
    dyT = dy.t().contiguous()
    xT = x.t().contiguous()
    fl = 2 * N * K * T
    t_nt = timeit(lambda: torch.mm(dy.t(), x, out=out))
    t_tn = timeit(lambda: torch.mm(dyT, xT.t(), out=out))
    t_tr = timeit(lambda: (dy.t().contiguous(), x.t().contiguous()))
    t_dx = timeit(lambda: torch.mm(dy, w))
    t_fw = timeit(lambda: torch.mm(x, w.t()))
    print(f"{name:5s} dW NT {t_nt:8.1f}us {fl / t_nt / 1e6:6.0f} TF | dW TN {t_tn:8.1f}us {fl / t_tn / 1e6:6.0f} TF "
          f"| transposes {t_tr:6.1f}us | dX {t_dx:7.1f}us {fl / t_dx / 1e6:6.0f} TF | fwd {t_fw:7.1f}us "
          f"{fl / t_fw / 1e6:6.0f} TF", flush=True)
