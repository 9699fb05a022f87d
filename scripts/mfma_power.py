"""FLOP per joule of the two bf16 MFMA shapes: runs build/mfma_power_probe (csrc/tests/mfma_power_probe.hip)
for each mode while sampling board power / sclk (scripts/power_probe.py's sampler).
    python scripts/mfma_power.py [seconds]
"""
import os
import subprocess
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from power_probe import Sampler, hwmons, ours, summarize  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    secs = sys.argv[1] if len(sys.argv) > 1 else "3"
    mons = ours(hwmons())
    smp = Sampler(mons)
    smp.start()
    exe = os.path.join(ROOT, "build", "mfma_power_probe")
    for mode in ("32", "16", "32", "16", "32z", "16z"):
        smp.samples = []
        time.sleep(0.3)
        p = subprocess.Popen([exe, mode, secs], stdout=subprocess.PIPE, text=True)
        time.sleep(0.8)  # skip the ramp
        smp.on = True
        out, _ = p.communicate()
        smp.on = False
        print(out.strip(), flush=True)
        summarize(f"  mfma {mode}", list(smp.samples), mons, 0.0)
    smp.stop_ = True


if __name__ == "__main__":
    torch.cuda.device_count()
    main()
