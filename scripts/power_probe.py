"""Is the 8B step power-bound? Board power and shader clock while the forward GEMM chain, the
flat AdamW, and both together run (the r2 finding: the two overlap to ~serial time even on
disjoint CUs, profiles/r1_cu_mask_overlap.log, r2_adamw_overlap_cap.log).

Samples the amdgpu hwmon sysfs files (power1_average / power1_input in uW, freq1_input = sclk in
Hz) from a host thread every 20 ms while each phase repeats its work for ~3 s.
    python scripts/power_probe.py
"""
import glob
import os
import sys
import threading
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fault_tolerant_llm_training_amd._native import kernels  # noqa: E402


def hwmons():
    out = []
    for h in sorted(glob.glob("/sys/class/drm/card*/device/hwmon/hwmon*")):
        files = {}
        for name in ("power1_average", "power1_input", "freq1_input", "freq2_input"):
            f = os.path.join(h, name)
            if os.path.exists(f):
                try:
                    open(f).read()
                    files[name] = f
                except OSError:
                    pass
        if files:
            out.append((h, files))
    return out


class Sampler(threading.Thread):
    def __init__(self, mons):
        super().__init__(daemon=True)
        self.mons, self.samples, self.on, self.stop_ = mons, [], False, False

    def run(self):
        while not self.stop_:
            if self.on:
                row = []
                for _, files in self.mons:
                    vals = {}
                    for k, f in files.items():
                        try:
                            vals[k] = int(open(f).read().strip())
                        except (OSError, ValueError):
                            pass
                    row.append(vals)
                self.samples.append(row)
            time.sleep(0.02)


def summarize(tag, samples, mons, ms):
    if not samples:
        print(f"{tag:28s} {ms:8.2f} ms/iter | no samples", flush=True)
        return
    parts = []
    for i, (h, _) in enumerate(mons):
        vals = [s[i] for s in samples if i < len(s)]
        pw = [v.get("power1_average", v.get("power1_input", 0)) / 1e6 for v in vals]
        sc = [v.get("freq1_input", 0) / 1e6 for v in vals]
        if max(pw, default=0) < 1 and max(sc, default=0) < 1:
            continue
        parts.append(f"{h.split('/')[4]}: "
                     f"power {sum(pw) / len(pw):6.0f} W (max {max(pw):5.0f}) sclk {sum(sc) / len(sc):6.0f} MHz "
                     f"(min {min(sc):5.0f})")
    print(f"{tag:28s} {ms:8.2f} ms/iter | " + " ; ".join(parts[:4]), flush=True)


def ours(mons):
    """The hwmon of cuda:0 (PCI address match), else every card."""
    pr = torch.cuda.get_device_properties(0)
    bus = getattr(pr, "pci_bus_id", None)
    if bus is None:
        return mons
    sel = []
    for h, f in mons:
        addr = os.path.basename(os.path.realpath(os.path.dirname(os.path.dirname(h))))
        try:
            b = int(addr.split(":")[1], 16)
        except (IndexError, ValueError):
            continue
        if b == bus:
            sel.append((h, f))
    print(f"cuda:0 pci bus {bus:#x} -> {[h for h, _ in sel]}", flush=True)
    return sel or mons


def main():
    mons = hwmons()
    print("hwmon:", [(h, os.path.realpath(os.path.dirname(os.path.dirname(h)))) for h, f in mons][:8], flush=True)
    torch.cuda.init()
    mons = ours(mons)
    K = kernels()
    dev = torch.device("cuda", 0)
    T, D, F = 2048, 4096, 14336
    x = (torch.rand(T, D, device=dev) * 2 - 1).bfloat16()
    ws = [((torch.rand(n, k, device=dev) * 2 - 1) * 0.02).bfloat16() for n, k in ((6144, D), (D, D), (2 * F, D), (D, F))]
    a = (torch.rand(T, F, device=dev) * 2 - 1).bfloat16()
    NP, NL = 7_500_000_000, 32
    p, g, m, v = (torch.empty(NP, dtype=torch.bfloat16, device=dev).normal_() for _ in range(4))
    stats = torch.tensor([1.0, 1.0, 0.0], device=dev)
    chunk = NP // NL
    s_g, s_o = torch.cuda.Stream(), torch.cuda.Stream()

    def gemms():
        with torch.cuda.stream(s_g):
            for _ in range(NL):
                torch.mm(x, ws[0].t())
                torch.mm(x, ws[1].t())
                torch.mm(x, ws[2].t())
                torch.mm(a, ws[3].t())

    def adamw():
        with torch.cuda.stream(s_o):
            for i in range(NL):
                sl = slice(i * chunk, (i + 1) * chunk)
                K.adamw_(p[sl], g[sl], m[sl], v[sl], stats, 1e-4, 0.9, 0.999, 1e-8, 0.01, 5, 0)

    smp = Sampler(mons)
    smp.start()

    def phase(tag, fns, secs=3.0):
        for f in fns:
            f()
        torch.cuda.synchronize()
        smp.samples = []
        smp.on = True
        n, t0 = 0, time.perf_counter()
        while time.perf_counter() - t0 < secs:
            for f in fns:
                f()
            torch.cuda.synchronize()
            n += 1
        dt = (time.perf_counter() - t0) / n * 1e3
        smp.on = False
        summarize(tag, list(smp.samples), mons, dt)

    time.sleep(0.5)
    phase("idle", [lambda: time.sleep(0.05)], 1.0)
    phase("gemm chain", [gemms])
    phase("adamw", [adamw])
    phase("gemm chain + adamw (2 str)", [gemms, adamw])
    phase("gemm chain", [gemms])
    if hasattr(K, "set_exact_math"):  # AdamW with IEEE division / sqrt vs the hardware rcp / sqrt
        for exact in (True, False, True, False):
            K.set_exact_math(exact)
            phase(f"adamw exact={int(exact)}", [adamw])
            phase(f"gemm chain + adamw exact={int(exact)}", [gemms, adamw])
        K.set_exact_math(False)
    smp.stop_ = True


if __name__ == "__main__":
    main()
