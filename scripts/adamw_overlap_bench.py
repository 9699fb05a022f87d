"""Does a bandwidth-capped AdamW overlap the forward GEMMs better than a full-grid one?

A Llama-3-8B-shaped forward GEMM chain (32 layers x {qkv, wo, w13, w2}, 2048 tokens) and a flat
bf16 AdamW over 8 B parameters in 32 per-layer launches, each alone and concurrently on two
streams (no CU masks), for AdamW grid caps (max_blocks; 0 = the default streaming grid).
    python scripts/adamw_overlap_bench.py
"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fault_tolerant_llm_training_amd._native import kernels  # noqa: E402

K = kernels()
dev = torch.device("cuda", 0)
T, D, F = 2048, 4096, 14336
x = (torch.rand(T, D, device=dev) * 2 - 1).bfloat16()
ws = [((torch.rand(n, k, device=dev) * 2 - 1) * 0.02).bfloat16() for n, k in ((6144, D), (D, D), (2 * F, D), (D, F))]
a = (torch.rand(T, F, device=dev) * 2 - 1).bfloat16()
NP, NL = 7_500_000_000, 32
p, g, m, v = (torch.empty(NP, dtype=torch.bfloat16, device=dev).normal_() for _ in range(4))
stats = torch.tensor([1.0, 1.0, 0.0], device=dev)
chunk = NP // NL
s_g, s_o = torch.cuda.Stream(), torch.cuda.Stream()


def gemms():
    with torch.cuda.stream(s_g):
        for _ in range(NL):
            torch.mm(x, ws[0].t())
            torch.mm(x, ws[1].t())
            torch.mm(x, ws[2].t())
            torch.mm(a, ws[3].t())


def adamw(cap):
    with torch.cuda.stream(s_o):
        for i in range(NL):
            sl = slice(i * chunk, (i + 1) * chunk)
            K.adamw_(p[sl], g[sl], m[sl], v[sl], stats, 1e-4, 0.9, 0.999, 1e-8, 0.01, 5, cap)


def timed(*fns, reps=3):
    best = 1e9
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for f in fns:
            f()
        torch.cuda.synchronize()
        best = min(best, time.perf_counter() - t0)
    return best * 1e3


gemms(); adamw(0); torch.cuda.synchronize()
tg = timed(gemms)
print(f"gemm chain alone {tg:7.2f} ms", flush=True)
for cap in (0, 2048, 1024, 512, 256, 128, 64):
    ta = timed(lambda: adamw(cap))
    to = timed(gemms, lambda: adamw(cap))
    print(f"adamw cap {cap:5d}: alone {ta:7.2f} ms ({14 * NP / ta / 1e9:5.2f} TB/s) | concurrent with gemms "
          f"{to:7.2f} ms | serial {tg + ta:7.2f} ms | hidden {100 * (tg + ta - to) / min(tg, ta):5.1f} % of the "
          f"shorter", flush=True)
