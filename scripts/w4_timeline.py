"""Per-workgroup exit times of the w4 GEMM (gemm_w4_set_prof: 100 MHz s_memrealtime after the
epilogue, and the CU) on the Llama-3-8B products: how long one tile takes on its CU (the gap
between consecutive exits on a CU = one tile + the dispatch of the next), how tightly the 256 CUs
move in step from round to round, and the kernel's tail.

Only the exit is stamped: any stamp before the K loop's drain changed the dW loops' code
(csrc/kernels/gemm_w4.h, probe_end).

    python scripts/w4_timeline.py
    FT_KERNELS_SO=probe/_kernels_probe.so python scripts/w4_timeline.py --full   (scripts/w4_probe_build.py)

--full: the investigation build also stamps the entry, the end of the prologue, the drain and the
end of the epilogue's LDS staging: prints the per-workgroup phase split and the gap between one
workgroup's exit and the next one's entry on the same CU.
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fault_tolerant_llm_training_amd._native import kernels  # noqa: E402

K_ = kernels()
r = lambda *s: (torch.rand(*s, device="cuda") * 2 - 1).bfloat16()  # noqa: E731


def timeit(fn, n=10, w=3):
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


FULL = "--full" in sys.argv


def phases(p):
    t0, t1, t2, t3, t7 = (p[:, i].astype(np.int64) for i in (0, 1, 2, 3, 7))
    pro, loop, stage, epi = (t1 - t0) / 100, (t2 - t1) / 100, (t7 - t2) / 100, (t3 - t7) / 100
    cu = (p[:, 5] << 16) | ((p[:, 4] >> 8) & 0xFF)
    gaps = []
    for c in set(cu.tolist()):
        m = cu == c
        iv = sorted(zip(t0[m].tolist(), t3[m].tolist()))
        gaps += [(b0 - a1) / 100 for (_, a1), (b0, _) in zip(iv, iv[1:])]
    f = lambda x: f"{np.mean(x):6.2f} (p10 {np.percentile(x, 10):6.2f} p90 {np.percentile(x, 90):6.2f})"  # noqa: E731
    print(f"    prologue {f(pro)} | K loop {f(loop)} | epilogue staging {f(stage)} | rest of epilogue {f(epi)} us"
          + (f" | exit -> next entry on the CU {f(gaps)} us" if gaps else ""), flush=True)


def probe(name, fn, grid):
    t_us = timeit(fn)
    buf = torch.zeros(grid, 8, dtype=torch.int64, device="cuda")
    K_.gemm_w4_set_prof(buf)
    fn()
    torch.cuda.synchronize()
    K_.gemm_w4_set_prof(None)
    p = buf.cpu().numpy()
    p = p[p[:, 3] != 0]
    if FULL:
        print(name, flush=True)
        phases(p)
    end = (p[:, 3] - p[:, 3].min()) / 100.0  # us after the first exit
    cu = (p[:, 5] << 16) | ((p[:, 4] >> 8) & 0xFF) | (((p[:, 4] >> 13) & 0x7) << 8)
    per_cu = {}
    for c, e in zip(cu.tolist(), end.tolist()):
        per_cu.setdefault(c, []).append(e)
    gaps = []
    for es in per_cu.values():
        es.sort()
        gaps += list(np.diff(es))
    first = np.array(sorted(es[0] for es in per_cu.values()))
    last = np.array(sorted(es[-1] for es in per_cu.values()))
    g = np.array(gaps) if gaps else np.zeros(1)
    nper = np.array([len(v) for v in per_cu.values()])
    print(f"{name:34s} {len(p):5d} WGs on {len(per_cu)} CUs ({nper.min()}-{nper.max()} each) | kernel {t_us:7.1f} us | "
          f"tile on a CU: mean {g.mean():6.2f} p10 {np.percentile(g, 10):6.2f} p90 {np.percentile(g, 90):6.2f} us | "
          f"first exits span {first[-1] - first[0]:5.2f} us, last exits span {last[-1] - last[0]:5.2f} us", flush=True)


def main():
    T, D, F, V = 2048, 4096, 14336, 131072
    for name, M, N, Kd, lay in (("wo fwd 2048x4096x4096 (1 round)", T, D, D, "fwd"),
                                ("w2 dW 4096x14336x2048", D, F, T, "dw"),
                                ("w13 dW 28672x4096x2048", 2 * F, D, T, "dw"),
                                ("qkv dW 6144x4096x2048", 6144, D, T, "dw"),
                                ("4096^2 x K=2048 fwd (1 round)", 4096, 4096, 2048, "fwd"),
                                ("4096^2 x K=2048 dw (1 round)", 4096, 4096, 2048, "dw"),
                                ("8192^2 x K=2048 dw (4 rounds)", 8192, 8192, 2048, "dw")):
        if lay == "fwd":
            a, b = r(M, Kd), r(N, Kd)
            nj = 8 if N % 256 == 0 and (M // 256) * (N // 256) >= 256 else 4
            fn = lambda: K_.gemm_nt_w4(a, b, None, None, nj, 1)  # noqa: E731
            grid = (M // 256) * (N // (32 * nj))
        else:
            a, b = r(Kd, M), r(Kd, N)
            fn = lambda: K_.gemm_w4_ex(a, True, b, True, M, N, Kd, None, False, None, 8, 1)  # noqa: E731
            grid = (M // 256) * (N // 256)
        probe(name, fn, grid)
        del a, b


if __name__ == "__main__":
    main()
