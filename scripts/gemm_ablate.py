"""Ablation timing of the hand GEMM main loop (forward NT layout), MI355X: full kernel vs
builds without the in-loop barrier (1), DMA (2), LDS reads (3), or with MFMAs only (4).
Results of 1-4 are wrong by construction; only the time matters. Random operands."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from fault_tolerant_llm_training_amd._native import kernels

K_ = kernels()
shapes = [(2048, 28672, 4096), (2048, 131072, 4096), (4096, 4096, 4096), (8192, 8192, 8192)]
names = {0: "full", 1: "no barrier", 2: "no DMA", 3: "no LDS read", 4: "MFMA only", 5: "no DMA wait", 6: "1-barrier sched"}
for M, N, Kd in shapes:
    a = (torch.rand(M, Kd, device="cuda") * 2 - 1).bfloat16()
    b = (torch.rand(N, Kd, device="cuda") * 2 - 1).bfloat16()
    fl = 2.0 * M * N * Kd
    res = {}
    for rnd in range(3):
        for abl in range(7):
            f = lambda: K_.gemm_ablate(a, b, M, N, Kd, abl)
            f()
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(5):
                f()
            e.record()
            torch.cuda.synchronize()
            res.setdefault(abl, []).append(s.elapsed_time(e) / 5 * 1e3)
    line = " | ".join(f"{names[k]} {min(v):7.1f} us {fl / min(v) / 1e6:5.0f} TF" for k, v in res.items())
    print(f"[{M}x{N}x{Kd}] {line}", flush=True)
