#!/usr/bin/env python3
"""Exports the kernel dispatches of a rocprofv3 SQLite database (``*_results.db``, the default output
format of this ROCm) to the CSV layout of ``--output-format csv`` that scripts/prof_summary.py and
scripts/prof_timeline.py read: ``<prefix>_kernel_trace.csv`` and ``<prefix>_kernel_stats.csv``.

    python scripts/rocpd_export.py gpurun_out/prof_r4/run_results.db [gpurun_out/prof_r4/run]
"""
import collections
import csv
import sqlite3
import sys


def main():
    db = sys.argv[1]
    prefix = sys.argv[2] if len(sys.argv) > 2 else db.rsplit("_results.db", 1)[0]
    c = sqlite3.connect(db)
    rows = c.execute("select name, stream_id, dispatch_id, start, end, grid_x, workgroup_x, lds_size, "
                     "scratch_size, vgpr_count, accum_vgpr_count, sgpr_count from kernels order by start").fetchall()
    with open(prefix + "_kernel_trace.csv", "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Kernel_Name", "Stream_Id", "Dispatch_Id", "Start_Timestamp", "End_Timestamp", "Grid_Size_X",
                    "Workgroup_Size_X", "LDS_Block_Size", "Scratch_Size", "VGPR_Count", "Accum_VGPR_Count",
                    "SGPR_Count"])
        w.writerows(rows)
    agg = collections.defaultdict(list)
    for r in rows:
        agg[r[0]].append(r[4] - r[3])
    total = sum(sum(v) for v in agg.values())
    with open(prefix + "_kernel_stats.csv", "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
        for name, d in sorted(agg.items(), key=lambda x: -sum(x[1])):
            w.writerow([name, len(d), sum(d), sum(d) / len(d), 100.0 * sum(d) / total, min(d), max(d)])
    print(f"{len(rows)} dispatches, {len(agg)} kernels -> {prefix}_kernel_trace.csv / _kernel_stats.csv")


if __name__ == "__main__":
    main()
