"""Loss curves of two train.py logs side by side ("Training step: N | Loss: X" lines), with the
largest difference and the mean difference over the last quarter of the run.
    python scripts/convergence_compare.py <title> <label_a> <log_a> <label_b> <log_b>
"""
import re
import sys

PAT = re.compile(r"Training step: (\d+) \| Loss: ([0-9.]+)")


def curve(path):
    out = {}
    with open(path) as f:
        for line in f:
            m = PAT.search(line)
            if m:
                out[int(m.group(1))] = float(m.group(2))
    return out


def main():
    title, la, pa, lb, pb = sys.argv[1:6]
    a, b = curve(pa), curve(pb)
    steps = sorted(set(a) & set(b))
    if not steps:
        sys.exit("no common logged steps")
    print(f"## {title}\n")
    print(f"| step | {la} | {lb} | diff |\n|---|---|---|---|")
    stride = max(1, len(steps) // 16)
    for s in steps[::stride] + ([steps[-1]] if steps[-1] not in steps[::stride] else []):
        print(f"| {s} | {a[s]:.4f} | {b[s]:.4f} | {a[s] - b[s]:+.4f} |")
    tail = steps[len(steps) * 3 // 4:]
    ma = sum(a[s] for s in tail) / len(tail)
    mb = sum(b[s] for s in tail) / len(tail)
    worst = max(abs(a[s] - b[s]) for s in steps)
    print(f"\nfirst logged loss {a[steps[0]]:.4f} / {b[steps[0]]:.4f}; last-quarter mean {ma:.4f} / {mb:.4f} "
          f"(diff {ma - mb:+.4f}); largest per-step difference {worst:.4f}\n")


if __name__ == "__main__":
    main()
