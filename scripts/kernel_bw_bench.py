#!/usr/bin/env python3
"""Bandwidth roofline of the memory-bound gfx950 kernels at the Llama-3-8B step shapes (MI355X).

Each kernel is timed alone (events, 20 launches after 3 warmups) and its compulsory HBM bytes
(every input read once, every output written once) divided by the time: the achieved fraction
of the ~6.3 TB/s a streaming copy reaches on MI355X (MI355X_MICROARCH.md) is the kernel's
distance from its speed of light.
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fault_tolerant_llm_training_amd._native import kernels  # noqa: E402
from fault_tolerant_llm_training_amd.models.llama import rope_tables  # noqa: E402

K = kernels()
T, D, F, V = 2048, 4096, 14336, 131072
Hq, Hkv, HD = 32, 8, 128
SOL = 6.3e12


def t(fn, it=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(it):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / it * 1e-3


def r(*shape):
    return torch.randn(*shape, device="cuda").bfloat16()


rows = []


def case(name, fn, nbytes):
    s = t(fn)
    rows.append((name, s * 1e6, nbytes / s / 1e12, nbytes / s / SOL))
    print(f"{name:34s} {s * 1e6:8.1f} us  {nbytes / s / 1e12:5.2f} TB/s  {100 * nbytes / s / SOL:5.1f} % of 6.3 TB/s",
          flush=True)


x, d, w = r(T, D), r(T, D), (1 + 0.1 * torch.randn(D, device="cuda")).bfloat16()
y, rstd, mean, h = K.add_norm_fwd(x, d, w, 1e-5, False)
case("add_norm_fwd [2048x4096]", lambda: K.add_norm_fwd(x, d, w, 1e-5, False), 4 * T * D * 2)
dy, dres, dw = r(T, D), r(T, D), torch.empty(D, device="cuda").bfloat16()
case("norm_bwd (+residual grad) [2048x4096]", lambda: K.norm_bwd(dy, h, w, rstd, None, dw, dres, False),
     4 * T * D * 2)
os.environ["FT_NORM_BWD_SPLIT"] = "0"  # A/B: the one-wave-per-row kernel
case("norm_bwd 1-wave-per-row (A/B)", lambda: K.norm_bwd(dy, h, w, rstd, None, dw, dres, False), 4 * T * D * 2)
os.environ.pop("FT_NORM_BWD_SPLIT")
case("norm_bwd split-row (again)", lambda: K.norm_bwd(dy, h, w, rstd, None, dw, dres, False), 4 * T * D * 2)
gu = r(T, 2 * F)
da = r(T, F)
qkv = r(T, (Hq + 2 * Hkv) * HD)
cos, sin = rope_tables(HD, T, 500000.0)
cos, sin = cos.cuda(), sin.cuda()
case("rope_fwd (q,k of packed qkv)", lambda: K.rope_fwd(qkv, cos, sin, T, Hq, Hkv, HD),
     2 * T * (Hq + Hkv) * HD * 2)
g2 = r(T, (Hq + 2 * Hkv) * HD)
case("rope_bwd_ (in place)", lambda: K.rope_bwd_(g2, cos, sin, T, Hq, Hkv, HD), 2 * T * (Hq + Hkv) * HD * 2)
logits = (3 * torch.randn(T, V, device="cuda")).bfloat16()
lab = torch.randint(0, V, (T,), device="cuda")
case("xent_fwd [2048x131072]", lambda: K.xent_fwd(logits, lab, -100), T * V * 2)
_, lse = K.xent_fwd(logits, lab, -100)
gg = torch.ones(1, device="cuda")
inv = torch.full((1,), 1.0 / T, device="cuda")
lg = logits.clone()
case("xent_bwd_ (dlogits in place)", lambda: K.xent_bwd_(lg, lab, lse, gg, inv, -100), 2 * T * V * 2)
n = 1 << 30
p, g, m, v = (torch.randn(n, device="cuda").bfloat16() for _ in range(4))
stats = torch.tensor([1.0, 1.0, 0.0], device="cuda")
case("adamw_ (1G params, bf16 p/g/m/v)", lambda: K.adamw_(p, g, m, v, stats, 1e-4, 0.9, 0.999, 1e-8, 0.01, 5, 0),
     14 * n)
part = torch.zeros(2048, device="cuda")
case("sumsq_into_ (1G bf16)", lambda: K.sumsq_into_(g, part), 2 * n)

print("\n| kernel | us | TB/s | % of 6.3 TB/s |\n|---|---|---|---|")
for name, us, tbs, frac in rows:
    print(f"| {name} | {us:.1f} | {tbs:.2f} | {100 * frac:.0f} |")
