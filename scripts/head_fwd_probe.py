"""LM-head logits GEMM at the GPT-2 sizes (K = 768 / 1024, V = 131072, 2048 tokens): the w4 kernel vs
the default route (mm_fwd), same process, medians of 3 x 30 launches.

    python scripts/head_fwd_probe.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fault_tolerant_llm_training_amd._native import kernels  # noqa: E402
from fault_tolerant_llm_training_amd.ops import functional as Fx  # noqa: E402


def t(fn, n=30):
    for _ in range(3):
        fn()
    e = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    e[0].record()
    for _ in range(n):
        fn()
    e[1].record()
    torch.cuda.synchronize()
    return e[0].elapsed_time(e[1]) / n * 1e3


def main():
    K_ = kernels()
    for D in (768, 1024):
        h = (torch.rand(2048, D, device="cuda") * 2 - 1).bfloat16()
        w = (torch.rand(131072, D, device="cuda") * 2 - 1).bfloat16()
        a = sorted(t(lambda: K_.gemm_nt_w4(h, w, None, None, 0)) for _ in range(3))[1]
        b = sorted(t(lambda: Fx.mm_fwd(h, w)) for _ in range(3))[1]
        f = 2 * 2048 * 131072 * D
        print(f"head fwd D={D}: w4 {a:.1f} us ({f / a / 1e6:.0f} TF/s) | mm_fwd {b:.1f} us ({f / b / 1e6:.0f} TF/s)",
              flush=True)


if __name__ == "__main__":
    main()
