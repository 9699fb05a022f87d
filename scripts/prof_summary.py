#!/usr/bin/env python3
"""Summarise a rocprofv3 ``*_kernel_stats.csv`` into a markdown table (for profiles/).

    python scripts/prof_summary.py gpurun_out/prof/run_kernel_stats.csv "title" [steps]
"""
import csv
import sys


def main():
    path, title = sys.argv[1], sys.argv[2]
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 0
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: -int(r["TotalDurationNs"]))
    total = sum(int(r["TotalDurationNs"]) for r in rows)
    print(f"# {title}\n")
    print(f"total GPU kernel time {total / 1e6:.1f} ms" + (f" over {steps} profiled steps "
          f"(incl. warmup) = {total / 1e6 / steps:.1f} ms/step" if steps else "") + "\n")
    print("| total ms | % | calls | avg us | kernel |\n|---|---|---|---|---|")
    for r in rows:
        t = int(r["TotalDurationNs"])
        name = r["Name"].replace("|", "/")
        if len(name) > 100:
            name = name[:100]
        print(f"| {t / 1e6:.2f} | {100 * t / total:.2f} | {r['Calls']} | {float(r['AverageNs']) / 1e3:.1f} | `{name}` |")


if __name__ == "__main__":
    main()
