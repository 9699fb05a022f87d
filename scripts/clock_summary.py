#!/usr/bin/env python3
"""Effective shader clock per kernel family from a rocprofv3 --pmc GRBM_GUI_ACTIVE run:
GRBM_GUI_ACTIVE is summed over the 8 XCDs, so clock = value / 8 / duration (MI355X_MICROARCH.md,
'DVFS give-back'; dispatches under ~0.3 ms read high, so only longer ones are counted).
    python scripts/clock_summary.py gpurun_out/clk/step/.../run_counter_collection.csv
"""
import collections
import csv
import statistics
import sys


def family(n: str) -> str:
    if "Cijk" in n:
        return "hipBLASLt GEMM"
    for k in ("adamw", "gemm_kernel", "flash_fwd", "flash_bwd", "sumsq", "norm", "swiglu", "transpose", "xent"):
        if k in n:
            return k
    return "other"


rows = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    if r["Counter_Name"] != "GRBM_GUI_ACTIVE":
        continue
    dur = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    if dur < 300_000:
        continue
    rows[family(r["Kernel_Name"])].append(float(r["Counter_Value"]) / 8 / dur)
for fam, v in sorted(rows.items(), key=lambda kv: -len(kv[1])):
    v.sort()
    print(f"{fam:16s} dispatches >= 0.3 ms: {len(v):4d}  clock GHz median {statistics.median(v):.2f}  "
          f"p10 {v[len(v) // 10]:.2f}  p90 {v[(9 * len(v)) // 10]:.2f}")
