"""Runs a few w4 GEMM products back to back for a rocprofv3 --pmc pass (LDS bank conflicts etc.):
the same output shape on the K-contiguous (forward) layout and on the k-major dX / dW layouts.

    rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --kernel-trace -d DIR -o NAME -- \
        python3 scripts/w4t_pmc_probe.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fault_tolerant_llm_training_amd._native import kernels  # noqa: E402


def main():
    K_ = kernels()
    r = lambda *s: (torch.rand(*s, device="cuda") * 2 - 1).bfloat16()
    M, N, Kd = 2048, 4096, 4096
    a, b, bt, at = r(M, Kd), r(N, Kd), r(Kd, N), r(Kd, M)
    for nj in (4, 8):
        for _ in range(3):
            K_.gemm_nt_w4(a, b, None, None, nj)                                   # forward layout
            K_.gemm_w4_ex(a, False, bt, True, M, N, Kd, None, False, None, nj)    # dX layout
            K_.gemm_w4_ex(at, True, bt, True, M, N, Kd, None, False, None, nj)    # dW layout
    torch.cuda.synchronize()
    print("done", flush=True)


if __name__ == "__main__":
    main()
