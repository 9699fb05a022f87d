"""Checkpoint writer throughput on this box's disk: the native O_DIRECT piece writer
(csrc/runtime/zip_writer.cpp) at several thread counts, 16 GiB from pinned host memory, fsync'd.
    python scripts/ckpt_write_bench.py [dir]
"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fault_tolerant_llm_training_amd._native import runtime  # noqa: E402

d = sys.argv[1] if len(sys.argv) > 1 else "/tmp/ft_write_bench"
os.makedirs(d, exist_ok=True)
rt = runtime()
GB = 16
buf = rt.pinned_empty(GB << 30)
buf.view(torch.int64).random_()
n = buf.numel()
piece = 1 << 30
offs = list(range(0, n, piece))
for threads in (4, 8, 16, 32, 8):
    path = os.path.join(d, "w.bin")
    with open(path, "wb") as f:
        f.truncate(n)
    t0 = time.perf_counter()
    rt.write_pieces(path, offs, [buf.data_ptr() + o for o in offs], [min(piece, n - o) for o in offs], threads, 0,
                    True, True)
    dt = time.perf_counter() - t0
    print(f"threads {threads:3d}: {GB} GiB in {dt:6.2f} s = {n / dt / 1e9:6.2f} GB/s (fsync'd, O_DIRECT)", flush=True)
    os.remove(path)
