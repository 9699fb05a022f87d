"""128 x 128-tile GEMM (gemm_nt_s, csrc/kernels/gemm_s.hip) vs hipBLASLt on the GPT-2-small /
-medium step products (T = 2048 tokens), graph-timed (20 calls per HIP graph, best of 5).

gemm_nt_s takes both operands K-contiguous, so every product is timed in that form:
  fwd  y  = x W^T      : A = x [T, K], B = W [N, K]                  (operands as they are)
  dX   dx = dy W       : A = dy [T, N], B = W^T [K, N]              (a transposed weight copy)
  dW   dW = dy^T x     : A = dy^T [N, T], B = x^T [K, T]            (transposed activations)
next to hipBLASLt in the layout the step uses (torch.mm on the row-major tensors).
    python scripts/gemm_s_bench.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from fault_tolerant_llm_training_amd._native import kernels  # noqa: E402

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


def main():
    tot = {}
    for tag, d, f, qkv, L in (("s", 768, 2048, 2304, 12), ("m", 1024, 2816, 3072, 24)):
        for name, N, Kd in (("qkv", qkv, d), ("wo", d, d), ("w13", 2 * f, d), ("w2", d, f)):
            x, w, dy = r(T, Kd), r(N, Kd), r(T, N)
            wT, dyT, xT = w.t().contiguous(), dy.t().contiguous(), x.t().contiguous()
            for kind, blas, a, b in (("fwd", lambda: torch.mm(x, w.t()), x, w),
                                     ("dX", lambda: torch.mm(dy, w), dy, wT),
                                     ("dW", lambda: torch.mm(dy.t(), x), dyT, xT)):
                ref = blas().float()
                out = K_.gemm_nt_s(a, b, None, None, 0)
                rel = ((out.float() - ref).norm() / ref.norm()).item()
                tb = graph_time(blas)
                ts = graph_time(lambda: K_.gemm_nt_s(a, b, None, None, 0))
                ts1 = graph_time(lambda: K_.gemm_nt_s(a, b, None, None, 1))
                M_, N_, K__ = a.shape[0], b.shape[0], a.shape[1]
                fl = 2 * M_ * N_ * K__
                best = min(ts, ts1)
                tot.setdefault(tag, [0.0, 0.0])
                tot[tag][0] += tb * L
                tot[tag][1] += min(best, tb) * L
                print(f"{tag} {kind:3s} {name:4s} [{M_:5d}x{N_:5d}x{K__:5d}] hipBLASLt {tb:6.1f} us "
                      f"({fl / tb / 1e6:5.0f} TF) | s auto-split {ts:6.1f} | s no-split {ts1:6.1f} us "
                      f"({fl / best / 1e6:5.0f} TF) | x{tb / best:4.2f} | rel {rel:.1e}", flush=True)
    for tag, (b, s) in tot.items():
        print(f"{tag}: per-step body GEMMs hipBLASLt {b / 1e3:.2f} ms, best-of {s / 1e3:.2f} ms")


if __name__ == "__main__":
    main()
