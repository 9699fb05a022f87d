"""Where a pipelined flash-forward block's time goes: per-block wall-clock stamps (entry, after the
prologue, after the key loop, after the stores; 100 MHz s_memrealtime) and the CU each block ran
on, from flash_set_fwd_prof.

    python scripts/flash_fwd_timeline.py [S Hq Hkv D [B]]

Prints the prologue / loop / epilogue split, the loop time per 64-key tile, how long the CUs sat
between blocks, and the kernel's span against the sum of its blocks' times.
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from fault_tolerant_llm_training_amd._native import kernels  # noqa: E402

K = kernels()
S, Hq, Hkv, D = (int(v) for v in sys.argv[1:5]) if len(sys.argv) >= 5 else (2048, 32, 8, 128)
Bt = int(sys.argv[5]) if len(sys.argv) >= 6 else 1
qkv = torch.randn(Bt * S, (Hq + 2 * Hkv) * D, device="cuda").bfloat16()
qk = torch.randn(Bt * S, (Hq + Hkv) * D, device="cuda").bfloat16()


def run():
    K.flash_set_fwd_split(0)
    buf = torch.zeros(2 * ((S + 127) // 128) * Bt * Hq, 8, dtype=torch.int64, device="cuda")
    for _ in range(5):
        K.flash_fwd(qk, qkv, S, Hq, Hkv, D)
    K.flash_set_fwd_prof(buf)
    K.flash_fwd(qk, qkv, S, Hq, Hkv, D)
    torch.cuda.synchronize()
    K.flash_set_fwd_prof(None)
    K.flash_set_fwd_split(-1)
    p = buf.cpu().numpy()
    p = p[p[:, 0] != 0]
    nblk = len(p)
    t0 = p[:, 0].min()
    us = lambda x: x / 100.0  # 100 MHz ticks -> us  # noqa: E731
    ent, pro, loop, end = (p[:, i] - t0 for i in range(4))
    hw, xcc, qt, nt = p[:, 4], p[:, 5], p[:, 6] >> 2, p[:, 7]
    cu = (xcc << 16) | ((hw >> 8) & 0xF) | (((hw >> 12) & 1) << 4) | (((hw >> 13) & 0x7) << 5)
    print(f"S={S} Hq={Hq} Hkv={Hkv} D={D} B={Bt}: {nblk} blocks on {len(set(cu.tolist()))} CUs, "
          f"span {us(end.max()):.1f} us")
    pro_t, loop_t, epi_t = us(pro - ent), us(loop - pro), us(end - loop)
    print(f"prologue  mean {pro_t.mean():6.2f} us  p10 {sorted(pro_t)[len(pro_t) // 10]:6.2f}  "
          f"p90 {sorted(pro_t)[9 * len(pro_t) // 10]:6.2f}")
    print(f"epilogue  mean {epi_t.mean():6.2f} us  p10 {sorted(epi_t)[len(epi_t) // 10]:6.2f}  "
          f"p90 {sorted(epi_t)[9 * len(epi_t) // 10]:6.2f}")
    # loop time against tile count (least squares): intercept = per-block loop overhead
    A = np.stack([nt, np.ones_like(nt)], 1).astype(float)
    (slope, icpt), *_ = np.linalg.lstsq(A, loop_t, rcond=None)
    print(f"key loop  {slope:6.3f} us per 64-key tile + {icpt:6.2f} us per block (fit over {nblk} blocks)")
    for q in sorted(set(qt.tolist()))[:: max(1, len(set(qt.tolist())) // 8)]:
        m = qt == q
        print(f"  q-tile {q:3d}: {int(nt[m].max()):3d} tiles  loop {loop_t[m].mean():7.2f} us  "
              f"total {us(end - ent)[m].mean():7.2f} us")
    # per CU: busy time (union of its blocks' intervals), first start, last end
    busy, idle_gap = [], []
    for c in sorted(set(cu.tolist())):
        m = cu == c
        iv = sorted(zip(ent[m].tolist(), end[m].tolist()))
        tot, cs, ce = 0, iv[0][0], iv[0][1]
        for a, b in iv[1:]:
            if a > ce:
                tot += ce - cs
                idle_gap.append(a - ce)
                cs, ce = a, b
            else:
                ce = max(ce, b)
        tot += ce - cs
        busy.append((us(tot), us(iv[0][0]), us(max(b for _, b in iv)), len(iv)))
    b = np.array(busy)
    print(f"per CU: busy {b[:, 0].mean():.1f} us mean (min {b[:, 0].min():.1f}, max {b[:, 0].max():.1f}); "
          f"first block starts {b[:, 1].mean():.2f} us mean (max {b[:, 1].max():.2f}); last end "
          f"mean {b[:, 2].mean():.1f} us (min {b[:, 2].min():.1f}); blocks/CU {b[:, 3].mean():.2f}")
    if idle_gap:
        print(f"  gaps with no block on a CU: {len(idle_gap)}, mean {us(np.mean(idle_gap)):.2f} us")
    conc = (us(end - ent)).sum() / (b[:, 0].sum())
    print(f"mean blocks resident while a CU is busy: {conc:.2f}")


run()
