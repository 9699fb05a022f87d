"""Can a memory-bound AdamW overlap compute-bound forward GEMMs if each gets its own CUs?

Times a Llama-3-8B-shaped forward GEMM chain (32 layers, 2048 tokens) and a flat AdamW
over 8 B bf16 parameters alone, serially, and concurrently on two streams, with the
optimizer stream restricted to k CUs (hipExtStreamCreateWithCUMask) and the GEMM stream
either unrestricted or on the complementary CUs.
"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fault_tolerant_llm_training_amd._native import kernels, runtime  # noqa: E402

K = kernels()
RT = runtime()
dev = torch.device("cuda", 0)
ncu = torch.cuda.get_device_properties(0).multi_processor_count
print("CUs", ncu, flush=True)
T, D, F = 2048, 4096, 14336
x = torch.randn(T, D, device=dev).bfloat16()
ws = [torch.randn(n, k, device=dev).bfloat16() * 0.02 for n, k in ((6144, D), (D, D), (2 * F, D), (D, F))]
a = torch.randn(T, F, device=dev).bfloat16()
NP = 8_000_000_000
NL = 32
p, g, m, v = (torch.empty(NP, dtype=torch.bfloat16, device=dev).normal_() for _ in range(4))
stats = torch.tensor([1.0, 1.0, 0.0], device=dev)
chunk = NP // NL


def gemms(stream):
    with torch.cuda.stream(stream):
        for _ in range(NL):
            torch.mm(x, ws[0].t())
            torch.mm(x, ws[1].t())
            torch.mm(x, ws[2].t())
            torch.mm(a, ws[3].t())


def adamw(stream):
    with torch.cuda.stream(stream):
        for i in range(NL):
            sl = slice(i * chunk, (i + 1) * chunk)
            K.adamw_(p[sl], g[sl], m[sl], v[sl], stats, 1e-4, 0.9, 0.999, 1e-8, 0.01, 5, 0)


def mask_words(cus):
    w = [0] * ((ncu + 31) // 32)
    for c in cus:
        w[c // 32] |= 1 << (c % 32)
    return w


def masked(cus):
    return torch.cuda.ExternalStream(RT.cu_mask_stream(0, mask_words(cus)), device=dev)


main = torch.cuda.current_stream()
side = torch.cuda.Stream()


def timed(fn, reps=3):
    best = 1e9
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        best = min(best, time.perf_counter() - t0)
    return best * 1e3


gemms(main); adamw(main); torch.cuda.synchronize()
tg = timed(lambda: gemms(main))
ta = timed(lambda: adamw(main))
print(f"gemm chain alone {tg:7.2f} ms | adamw alone {ta:7.2f} ms | serial {tg + ta:7.2f} ms", flush=True)
print(f"unmasked 2-stream overlap {timed(lambda: (gemms(main), adamw(side))):7.2f} ms", flush=True)
for k in (16, 32, 48, 64, 96):
    for layout in ("spread", "block"):
        if layout == "spread":
            cus = [int(i * ncu / k) for i in range(k)]
        else:
            cus = list(range(ncu - k, ncu))
        rest = [c for c in range(ncu) if c not in set(cus)]
        so, sg = masked(cus), masked(rest)
        tak = timed(lambda: adamw(so))
        tgr = timed(lambda: gemms(sg))
        both = timed(lambda: (gemms(main), adamw(so)))
        both_c = timed(lambda: (gemms(sg), adamw(so)))
        print(f"k={k:3d} {layout:6s} adamw@k {tak:7.2f} | gemm@rest {tgr:7.2f} | overlap gemm(all) {both:7.2f}"
              f" | overlap gemm(rest) {both_c:7.2f}", flush=True)
