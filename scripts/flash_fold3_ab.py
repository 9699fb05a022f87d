"""GQA deterministic flash backward: 3 kernels (dK/dV first with its own delta, then dQ + the GQA
fold; flash_set_fold3(True)) vs 4 (dQ, dK/dV, finalize; the default), same process, alternating, at the
Llama-3-8B layer (S = 2048, 32 / 8 heads of 128, RoPE tables as in the step).

    python scripts/flash_fold3_ab.py [S Hq Hkv D]
    FOLD3_ONLY=0|1 python scripts/flash_fold3_ab.py   (one form only: for a per-kernel trace)
"""
import os
import sys

import torch

sys.path.insert(0, os.getcwd())
from fault_tolerant_llm_training_amd._native import kernels  # noqa: E402
from fault_tolerant_llm_training_amd.models.llama import rope_tables  # noqa: E402

K = kernels()
S, Hq, Hkv, D = (int(v) for v in sys.argv[1:5]) if len(sys.argv) >= 5 else (2048, 32, 8, 128)
qkv = torch.randn(S, (Hq + 2 * Hkv) * D, device="cuda").bfloat16()
qk = torch.randn(S, (Hq + Hkv) * D, device="cuda").bfloat16()
do = torch.randn(S, Hq * D, device="cuda").bfloat16()
cos, sin = (t.cuda() for t in rope_tables(D, S, 500000.0))
o, lse = K.flash_fwd(qk, qkv, S, Hq, Hkv, D)


def t(it=50):
    f = lambda: K.flash_bwd(do, qk, qkv, o, lse, S, Hq, Hkv, D, 1, cos, sin)  # noqa: E731
    for _ in range(5):
        f()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(it):
        f()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / it * 1e3


only = os.environ.get("FOLD3_ONLY")
forms = (True, False) if only is None else (only == "1",)
res = {True: [], False: []}
for r in range(5):
    for on in forms:
        K.flash_set_fold3(on)
        res[on].append(t())
K.flash_set_fold3(False)
unit = 2 * (S * S / 2) * D * Hq
for on in forms:
    b = min(res[on])
    print(f"{'3 kernels (fold in dQ)' if on else '4 kernels (finalize)':24s} best {b:7.1f} us  "
          f"{5 * unit / b / 1e6:5.0f} TF/s  all {' '.join(f'{x:.1f}' for x in res[on])}", flush=True)
