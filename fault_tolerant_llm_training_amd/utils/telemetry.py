"""Board telemetry of the GPU this rank drives: power, shader clock, power cap.

The Llama-3-8B step runs at the MI355X board power limit (docs/PERFORMANCE.md), so its step time
is set by energy per step and by how hard the box's firmware clocks down at that limit — which
differs box to box by a few percent. ``bench.py`` samples the amdgpu hwmon files (the same files
``scripts/power_probe.py`` reads) on a host thread over the timed region and reports the
median power and shader clock next to the step time, so a slower number can be told apart from
a hotter / lower-clocked box.

    power1_average / power1_input   board power, microwatts
    power1_cap                      power limit, microwatts
    freq1_input                     shader clock (sclk), Hz

Nothing here touches the GPU: it reads sysfs only (missing files → fields are None).
"""
from __future__ import annotations

import glob
import os
import threading
import time
from typing import Dict, List, Optional


def _read_int(path: str) -> Optional[int]:
    try:
        with open(path) as f:
            return int(f.read().strip())
    except (OSError, ValueError):
        return None


def hwmon_for_pci_bus(bus: Optional[int]) -> Optional[str]:
    """The hwmon directory of the amdgpu card on PCI bus ``bus`` (None: the first card with power)."""
    cands = []
    for h in sorted(glob.glob("/sys/class/drm/card*/device/hwmon/hwmon*")):
        if not (os.path.exists(os.path.join(h, "power1_average")) or os.path.exists(os.path.join(h, "power1_input"))):
            continue
        addr = os.path.basename(os.path.realpath(os.path.dirname(os.path.dirname(h))))
        try:
            b = int(addr.split(":")[1], 16)
        except (IndexError, ValueError):
            b = None
        cands.append((h, b))
    if not cands:
        return None
    if bus is not None:
        for h, b in cands:
            if b == bus:
                return h
    return cands[0][0]


class PowerSampler(threading.Thread):
    """Samples power and sclk every ``period_s`` while ``on`` is set."""

    def __init__(self, hwmon: Optional[str], period_s: float = 0.02):
        super().__init__(daemon=True)
        self.hwmon = hwmon
        self.period_s = period_s
        self.on = False
        self.stop_ = False
        self.power_w: List[float] = []
        self.sclk_mhz: List[float] = []
        p = None
        if hwmon:
            for name in ("power1_average", "power1_input"):
                if os.path.exists(os.path.join(hwmon, name)):
                    p = os.path.join(hwmon, name)
                    break
        self._pfile = p
        self._ffile = os.path.join(hwmon, "freq1_input") if hwmon else None

    def run(self) -> None:
        if self._pfile is None:
            return
        while not self.stop_:
            if self.on:
                pw = _read_int(self._pfile)
                fq = _read_int(self._ffile) if self._ffile else None
                if pw is not None:
                    self.power_w.append(pw / 1e6)
                if fq is not None:
                    self.sclk_mhz.append(fq / 1e6)
            time.sleep(self.period_s)

    def power_cap_w(self) -> Optional[float]:
        if not self.hwmon:
            return None
        v = _read_int(os.path.join(self.hwmon, "power1_cap"))
        return None if v is None else v / 1e6

    def summary(self) -> Dict[str, Optional[float]]:
        def q(xs, f):
            if not xs:
                return None
            s = sorted(xs)
            return round(s[min(len(s) - 1, int(f * len(s)))], 1)

        return {
            "power_w_p50": q(self.power_w, 0.5),
            "power_w_p10": q(self.power_w, 0.1),
            "power_w_p90": q(self.power_w, 0.9),
            "sclk_mhz_p50": q(self.sclk_mhz, 0.5),
            "sclk_mhz_p10": q(self.sclk_mhz, 0.1),
            "power_cap_w": self.power_cap_w(),
            "telemetry_samples": len(self.power_w),
        }


def start_sampler(device_index: int = 0) -> Optional[PowerSampler]:
    """A started (idle) sampler for ``cuda:device_index``'s board, or None when there is no hwmon."""
    try:
        import torch

        bus = getattr(torch.cuda.get_device_properties(device_index), "pci_bus_id", None)
    except Exception:  # noqa: BLE001 - telemetry is best effort
        bus = None
    h = hwmon_for_pci_bus(bus)
    if h is None:
        return None
    s = PowerSampler(h)
    s.start()
    return s
