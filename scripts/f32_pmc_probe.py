"""PMC probe of the fp32 GEMM: the 8B w1|w3 forward (2048 x 28672 x 4096) on gemm_f32 and on
hipBLASLt (torch.mm), 3 launches each. Run under rocprofv3 --pmc --kernel-trace; --summary DIR
prints the mean counters per kernel family.
"""
import csv
import glob
import os
import sys
from collections import defaultdict


def run():
    import torch

    sys.path.insert(0, os.getcwd())
    from fault_tolerant_llm_training_amd._native import kernels

    K_ = kernels()
    M, N, Kd = 2048, 28672, 4096
    a = torch.rand(M, Kd, device="cuda")
    b = torch.rand(N, Kd, device="cuda")
    for _ in range(3):
        K_.gemm_f32(a, False, b, False, M, N, Kd)
    for _ in range(3):
        torch.mm(a, b.t())
    torch.cuda.synchronize()


def summary(d):
    rows = defaultdict(lambda: defaultdict(float))
    names = {}
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            i = int(r["Dispatch_Id"])
            names[i] = r["Kernel_Name"]
            rows[i][r["Counter_Name"]] += float(r["Counter_Value"])
    fam = defaultdict(list)
    for i in sorted(rows):
        fam["gemm_f32" if "gemm_f32" in names[i] else names[i][:60]].append(i)
    for k, ids in fam.items():
        print(k, f"({len(ids)} launches)")
        for c in sorted({c for i in ids for c in rows[i]}):
            print(f"   {c:28s} {sum(rows[i][c] for i in ids) / len(ids):18.0f}")
        r0 = rows[ids[0]]
        if r0.get("SQ_BUSY_CYCLES") and "SQ_VALU_MFMA_BUSY_CYCLES" in r0:
            v = sum(rows[i]["SQ_VALU_MFMA_BUSY_CYCLES"] for i in ids) / sum(rows[i]["SQ_BUSY_CYCLES"] for i in ids)
            print(f"   MFMA busy / SQ busy          {v:18.3f}")


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--summary":
        summary(sys.argv[2])
    else:
        run()
