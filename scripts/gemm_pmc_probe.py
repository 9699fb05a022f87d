"""One GEMM shape, hand kernel and hipBLASLt, for rocprofv3 --pmc passes (scripts/gpu_pmc.sh).
    python scripts/gemm_pmc_probe.py [M N K [fwd|dw]]   (default: the 8B w13 forward, 2048 x 28672 x 4096)
dw: the weight-gradient layout (dY^T X from row-major dY [K, M] and X [K, N]); FT_GEMM_ASM_READS
selects the hand kernel's fragment reads (asm / builtin).
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fault_tolerant_llm_training_amd._native import kernels  # noqa: E402

M, N, K = (int(v) for v in sys.argv[1:4]) if len(sys.argv) >= 4 else (2048, 28672, 4096)
layout = sys.argv[4] if len(sys.argv) >= 5 else "fwd"
k = kernels()
if layout == "w4":  # the 4-wave kernel (csrc/kernels/gemm_w4.hip) vs hipBLASLt, forward layout
    var = int(os.environ.get("FT_W4_VARIANT", "3"))
    a = (torch.rand(M, K, device="cuda") * 2 - 1).bfloat16()
    b = (torch.rand(N, K, device="cuda") * 2 - 1).bfloat16()
    for _ in range(20):
        k.gemm_nt_w4(a, b, None, None, var)
        torch.mm(a, b.t())
elif layout == "dw":
    a = (torch.rand(K, M, device="cuda") * 2 - 1).bfloat16()
    b = (torch.rand(K, N, device="cuda") * 2 - 1).bfloat16()
    for _ in range(20):
        k.gemm(a, False, b, False, M, N, K, None, None, False, 1)
        torch.mm(a.t(), b)
else:
    a = (torch.rand(M, K, device="cuda") * 2 - 1).bfloat16()
    b = (torch.rand(N, K, device="cuda") * 2 - 1).bfloat16()
    for _ in range(20):
        k.gemm(a, True, b, True, M, N, K, None, None, False, 1)
        torch.mm(a, b.t())
torch.cuda.synchronize()
