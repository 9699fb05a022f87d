"""Times the deterministic flash backward at the 8B layer shape with the GQA fold in the dK/dV kernel
vs the finalize pass (and, via FT_FLASH_FOLD_DBG, the fold's parts).

    FT_FLASH_FOLD_DBG=0|1|2 python scripts/flash_fold_probe.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fault_tolerant_llm_training_amd._native import kernels  # noqa: E402
from fault_tolerant_llm_training_amd.models.llama import rope_tables  # noqa: E402


def main():
    K = kernels()
    S, Hq, Hkv, D = 2048, 32, 8, 128
    torch.manual_seed(0)
    qkv = torch.randn(S, (Hq + 2 * Hkv) * D, device="cuda").bfloat16()
    qk = qkv
    do = torch.randn(S, Hq * D, device="cuda").bfloat16()
    cos, sin = (t.cuda() for t in rope_tables(D, S, 500000.0))
    o, lse = K.flash_fwd(qk, qkv, S, Hq, Hkv, D)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    for fold in (False, True, False, True):
        K.flash_set_bwd_fold(fold)
        for _ in range(5):
            K.flash_bwd(do, qk, qkv, o, lse, S, Hq, Hkv, D, 1, cos, sin)
        ev[0].record()
        for _ in range(50):
            K.flash_bwd(do, qk, qkv, o, lse, S, Hq, Hkv, D, 1, cos, sin)
        ev[1].record()
        torch.cuda.synchronize()
        print(f"fold={fold} dbg={os.environ.get('FT_FLASH_FOLD_DBG', '0')}: {ev[0].elapsed_time(ev[1]) / 50 * 1e3:.1f} us",
              flush=True)
    K.flash_set_bwd_fold(True)


if __name__ == "__main__":
    main()
