"""PMC probe of the grouped tile raster: the 8B w1|w3 dW product (28672 x 4096 x 2048) with the
plain raster (group 0) and the default 8 x 4 blocks, 5 launches each (the first 2 of each as
warm-up). Run under rocprofv3 --pmc (scripts/gpu_pmc.sh style); the w4 dispatches come in that
order, so the summary takes dispatches 2-4 as group 0 and 7-9 as group 8.

    rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum ... -- python3 scripts/w4_raster_pmc_probe.py
    python scripts/w4_raster_pmc_probe.py --summary <pmc dir>
"""
import csv
import glob
import os
import sys
from collections import defaultdict


def run():
    import torch

    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from fault_tolerant_llm_training_amd._native import kernels

    K_ = kernels()
    M, N, Kd = 28672, 4096, 2048
    a = (torch.rand(Kd, M, device="cuda") * 2 - 1).bfloat16()
    b = (torch.rand(Kd, N, device="cuda") * 2 - 1).bfloat16()
    out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    part = torch.empty((M // 256) * (N // 128), device="cuda")
    for g in (0, 8):
        K_.gemm_w4_set_group(g)
        for _ in range(5):
            K_.gemm_w4_ex(a, True, b, True, M, N, Kd, out, False, part, 0)
        torch.cuda.synchronize()
    K_.gemm_w4_set_group(-1)


def summary(d):
    rows = defaultdict(dict)
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "gemm_w4_kernel" not in r["Kernel_Name"]:
                continue
            rows[int(r["Dispatch_Id"])][r["Counter_Name"]] = rows[int(r["Dispatch_Id"])].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    ids = sorted(rows)
    if len(ids) < 10:
        print(f"expected 10 w4 dispatches, got {len(ids)}")
        return
    for name, sel in (("group 0 (plain raster)", ids[2:5]), ("group 8 (8 x 4 blocks)", ids[7:10])):
        cs = sorted({c for i in sel for c in rows[i]})
        print(name)
        for c in cs:
            v = sum(rows[i].get(c, 0.0) for i in sel) / len(sel)
            print(f"   {c:28s} {v:18.0f}")
        if "TCC_HIT_sum" in cs and "TCC_MISS_sum" in cs:
            h = sum(rows[i]["TCC_HIT_sum"] for i in sel)
            m = sum(rows[i]["TCC_MISS_sum"] for i in sel)
            print(f"   L2 hit rate                  {h / (h + m):18.3f}")


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--summary":
        summary(sys.argv[2])
    else:
        run()
