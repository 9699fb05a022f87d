"""HBM bandwidth ceilings vs the flat AdamW / sum-of-squares kernels (1 GiB-element buffers)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fault_tolerant_llm_training_amd._native import kernels  # noqa: E402

K = kernels()
n = 1 << 30  # elements (bf16): 2 GiB per buffer
p, g, m, v = (torch.randn(n, device="cuda").bfloat16() for _ in range(4))
stats = torch.tensor([1.0, 1.0, 0.0], device="cuda")
dst = torch.empty_like(p)


def t(fn, it=10):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(it):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / it * 1e-3


s = t(lambda: dst.copy_(p))
print(f"torch copy      {2 * 2 * n / s / 1e12:6.2f} TB/s", flush=True)
part = torch.zeros(2048, device="cuda")
s = t(lambda: K.sumsq_into_(g, part))
print(f"sumsq           {2 * n / s / 1e12:6.2f} TB/s", flush=True)
for blocks in (0, 4096, 8192, 16384, 65535):
    s = t(lambda: K.adamw_(p, g, m, v, stats, 1e-4, 0.9, 0.999, 1e-8, 0.01, 5, blocks))
    print(f"adamw blocks={blocks:6d} {14 * n / s / 1e12:6.2f} TB/s  ({s * 1e3:.2f} ms per 1G params)", flush=True)
