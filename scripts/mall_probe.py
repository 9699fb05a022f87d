"""Does a gradient read straight after the GEMM that wrote it come from the 256 MB Infinity Cache
(MALL)? Times the grad-norm partial-sum kernel (sumsq_into_) over a bf16 buffer of one
Llama-3-8B weight-gradient size right after writing it (warm) vs after 1 GiB of other writes
(cold). If warm reads run much faster, a per-parameter sum of squares launched right behind each
dW GEMM reads cache instead of HBM (the per-bucket pass reads 16 GB of HBM per step).
    python scripts/mall_probe.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fault_tolerant_llm_training_amd._native import kernels  # noqa: E402


def main():
    K = kernels()
    dev = torch.device("cuda", 0)
    other = torch.empty(512 * 2**20, dtype=torch.bfloat16, device=dev)  # 1 GiB
    part = torch.zeros(2048, dtype=torch.float32, device=dev)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    for name, n in (("wo 4096x4096", 4096 * 4096), ("w2 4096x14336", 4096 * 14336),
                    ("w13 28672x4096", 28672 * 4096), ("bucket 256 MiB", 128 * 2**20)):
        g = torch.empty(n, dtype=torch.bfloat16, device=dev)
        res = {}
        for mode in ("cold", "warm", "cold", "warm"):
            ts = []
            for _ in range(5):
                if mode == "cold":
                    g.fill_(0.5)
                    other.fill_(0.25)
                else:
                    other.fill_(0.25)
                    g.fill_(0.5)
                ev[0].record()
                K.sumsq_into_(g, part)
                ev[1].record()
                torch.cuda.synchronize()
                ts.append(ev[0].elapsed_time(ev[1]) * 1e3)
            res.setdefault(mode, []).append(sorted(ts)[len(ts) // 2])
        gb = n * 2 / 1e9
        c, w = min(res["cold"]), min(res["warm"])
        print(f"{name:16s} {gb * 1e3:7.0f} MB  cold {c:7.1f} us ({gb / c * 1e6 / 1e3:5.2f} TB/s)  "
              f"warm {w:7.1f} us ({gb / w * 1e6 / 1e3:5.2f} TB/s)  warm/cold {w / c:.2f}", flush=True)


if __name__ == "__main__":
    main()
