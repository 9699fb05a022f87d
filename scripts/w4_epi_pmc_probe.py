"""PMC probe of the w4 epilogue staging writes: the Llama-3-8B products of every epilogue form
(plain dW with sum-of-squares partials, plain forward, fused SwiGLU forward with a^T, fused SwiGLU
backward, residual), 5 launches each, the first 2 of each as warm-up. Run under rocprofv3 --pmc
(one pass per counter set, kernel-trace only), then summarise per product:

    rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE -d DIR -o run \\
        --output-format csv -- python3 scripts/w4_epi_pmc_probe.py
    python scripts/w4_epi_pmc_probe.py --summary DIR
"""
import csv
import glob
import os
import sys
from collections import defaultdict

NAMES = ["w13 dW (k-major, partials)", "w2 fwd (plain)", "w13 fwd (SwiGLU + a^T)", "w2 dX (SwiGLU bwd)",
         "wo fwd (residual)"]
REPS = 5


def run():
    import torch

    # the tree to measure: the working directory's (an A/B worktree runs this file from its own root)
    sys.path.insert(0, os.getcwd())
    from fault_tolerant_llm_training_amd._native import kernels

    K_ = kernels()
    T, D, F = 2048, 4096, 14336
    r = lambda *s: (torch.rand(*s, device="cuda") * 2 - 1).bfloat16()
    xt, dgu = r(T, D), r(T, 2 * F)  # dW: (x^T)^T-layout operands, K = tokens
    part = torch.empty(((2 * F) // 256) * (D // 128) * 4, device="cuda")
    x, w2, a, w13, wo = r(T, D), r(D, F), r(T, F), r(2 * F, D) * 0.02, r(D, D)
    dy, gu, res = r(T, D), r(T, 2 * F), r(T, D)
    prods = [
        lambda: K_.gemm_w4_ex(dgu, True, xt, True, 2 * F, D, T, None, False, part, 0),
        lambda: K_.gemm_nt_w4(a, w2, None, None, 0, 0),
        lambda: K_.gemm_swiglu_w4(x, w13, True),
        lambda: K_.gemm_swiglu_bwd_w4(dy, w2, gu, 0),
        lambda: K_.gemm_nt_w4(x, wo, None, res, 0, 0),
    ]
    for f in prods:
        for _ in range(REPS):
            f()
        torch.cuda.synchronize()
    print("done", flush=True)


def summary(d):
    rows = defaultdict(dict)
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "gemm_w4_kernel" not in r["Kernel_Name"]:
                continue
            i = int(r["Dispatch_Id"])
            rows[i][r["Counter_Name"]] = rows[i].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    ids = sorted(rows)
    if len(ids) != REPS * len(NAMES):
        print(f"expected {REPS * len(NAMES)} w4 dispatches, got {len(ids)}")
        return
    for p, name in enumerate(NAMES):
        sel = ids[p * REPS + 2:(p + 1) * REPS]
        cs = sorted({c for i in sel for c in rows[i]})
        print(name)
        for c in cs:
            v = sum(rows[i].get(c, 0.0) for i in sel) / len(sel)
            print(f"   {c:28s} {v:18.0f}")
        if "SQ_LDS_BANK_CONFLICT" in cs and "SQ_INSTS_LDS" in cs:
            bc = sum(rows[i]["SQ_LDS_BANK_CONFLICT"] for i in sel)
            li = sum(rows[i]["SQ_INSTS_LDS"] for i in sel)
            print(f"   bank-conflict cycles / LDS instructions {bc / li:8.4f}")


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--summary":
        summary(sys.argv[2])
    else:
        run()
