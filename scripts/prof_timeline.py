#!/usr/bin/env python3
"""Timeline view of a rocprofv3 ``*_kernel_trace.csv``: busy/idle/overlap of the last N steps.

    python scripts/prof_timeline.py gpurun_out/prof/run_kernel_trace.csv [--steps 3]

A step boundary is taken at each launch of the cross-entropy forward kernel (one per step).
Reports, for the last ``--steps`` steps: wall time, time with >= 1 kernel running (busy),
idle gaps (count, total, largest), time with >= 2 kernels running concurrently, kernel time
per queue, and the kernel time per kernel family, so stalls between kernels and the
optimizer/compute overlap are visible.
"""
from __future__ import annotations

import argparse
import csv
import re
from collections import defaultdict


def family(name: str) -> str:
    if name.startswith("Cijk") or name.startswith("Custom_Cijk"):
        return "gemm(hipBLASLt)"
    m = re.search(r"gemm_w4_kernel<\w+, (\d+), (\d+), (\w+), (\w+)>", name)
    if m:  # NJ, epilogue, k-major A, k-major B
        lay = {("false", "false"): "fwd", ("false", "true"): "dX", ("true", "true"): "dW"}.get((m.group(3), m.group(4)), "?")
        return f"gemm_w4 {lay} nj{m.group(1)} epi{m.group(2)}"
    m = re.search(r"\(anonymous namespace\)::(\w+)", name)
    if m:
        return m.group(1)
    m = re.search(r"at::native::[^(]*?(\w+_kernel\w*)", name)
    if m:
        return "torch:" + m.group(1)
    return name[:40]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--marker", default="xent_fwd_kernel")
    a = ap.parse_args()
    ks = []
    for r in csv.DictReader(open(a.trace)):
        ks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r.get("Queue_Id", "?")))
    ks.sort()
    marks = [s for s, _, n, _ in ks if a.marker in n]
    if len(marks) < a.steps + 1:
        print(f"only {len(marks)} step markers found")
        return
    t0, t1 = marks[-a.steps - 1], marks[-1]
    win = [(max(s, t0), min(e, t1), n, q) for s, e, n, q in ks if e > t0 and s < t1]
    wall = t1 - t0
    ev = []
    for s, e, _, _ in win:
        ev += [(s, 1), (e, -1)]
    ev.sort()
    busy = conc = 0
    gaps = []
    depth, last = 0, t0
    for t, d in ev:
        if depth >= 1:
            busy += t - last
        if depth >= 2:
            conc += t - last
        if depth == 0 and t > last:
            gaps.append(t - last)
        depth += d
        last = t
    if t1 > last:
        gaps.append(t1 - last)
    fam = defaultdict(lambda: [0, 0])
    queues = defaultdict(int)
    for s, e, n, q in win:
        fam[family(n)][0] += e - s
        fam[family(n)][1] += 1
        queues[q] += e - s
    n = a.steps
    print(f"steps {n}: wall {wall / 1e6 / n:.2f} ms/step | busy {busy / 1e6 / n:.2f} | idle {(wall - busy) / 1e6 / n:.2f} "
          f"({len(gaps) / n:.0f} gaps/step, largest {max(gaps, default=0) / 1e3:.0f} us) | "
          f">=2 kernels running {conc / 1e6 / n:.2f} ms/step")
    print("kernel ms/step per queue: " + ", ".join(f"q{q}: {t / 1e6 / n:.1f}" for q, t in sorted(queues.items())))
    print("\n| family | kernel ms/step | calls/step |\n|---|---|---|")
    for f, (t, c) in sorted(fam.items(), key=lambda x: -x[1][0]):
        print(f"| {f} | {t / 1e6 / n:.2f} | {c / n:.0f} |")


if __name__ == "__main__":
    main()
