"""Flash attention fwd / bwd timing on the Llama-3-8B layer shape (B=1, S=2048, 32/8 heads, d=128)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from fault_tolerant_llm_training_amd._native import kernels

K = kernels()
# python scripts/flash_bench.py [S Hq Hkv D [B]]  (default: the Llama-3-8B layer, S=2048, 32/8 heads, d=128)
S, Hq, Hkv, D = (int(v) for v in sys.argv[1:5]) if len(sys.argv) >= 5 else (2048, 32, 8, 128)
Bt = int(sys.argv[5]) if len(sys.argv) >= 6 else 1
print(f"S={S} Hq={Hq} Hkv={Hkv} D={D}" + (f" B={Bt}" if Bt > 1 else ""))
qkv = torch.randn(Bt * S, (Hq + 2 * Hkv) * D, device="cuda").bfloat16()
qk = torch.randn(Bt * S, (Hq + Hkv) * D, device="cuda").bfloat16()
do = torch.randn(Bt * S, Hq * D, device="cuda").bfloat16()
o, lse = K.flash_fwd(qk, qkv, S, Hq, Hkv, D)
unit = 2 * (S * S / 2) * D * Hq * Bt  # flops of one causal [S x S/2 x D] matmul over all heads


def t(fn, it=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(it):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / it * 1e3


tf = t(lambda: K.flash_fwd(qk, qkv, S, Hq, Hkv, D))
print(f"fwd {tf:7.1f} us  {2 * unit / tf / 1e6:6.0f} TF/s")
if hasattr(K, "flash_set_fwd_split"):  # forward key split forced off / on (default: auto)
    for v in (0, 1):
        K.flash_set_fwd_split(v)
        tf = t(lambda: K.flash_fwd(qk, qkv, S, Hq, Hkv, D))
        print(f"fwd key split {'on ' if v else 'off'} {tf:7.1f} us  {2 * unit / tf / 1e6:6.0f} TF/s")
    K.flash_set_fwd_split(-1)
if hasattr(K, "flash_set_fwd_pipe"):  # software-pipelined forward off / on (default: on)
    for v, name in ((0, "unpipelined"), (1, "pipelined")):
        K.flash_set_fwd_pipe(v)
        tf = t(lambda: K.flash_fwd(qk, qkv, S, Hq, Hkv, D))
        print(f"fwd {name:26s} {tf:7.1f} us  {2 * unit / tf / 1e6:6.0f} TF/s")
    K.flash_set_fwd_pipe(1)
for mode, name in ((0, "bwd atomics"), (1, "bwd deterministic"), (2, "bwd no-atomic (racy, timing only)")):
    tb = t(lambda: K.flash_bwd(do, qk, qkv, o, lse, S, Hq, Hkv, D, mode))
    print(f"{name:34s} {tb:7.1f} us  {5 * unit / tb / 1e6:6.0f} TF/s (5-matmul count)")
if hasattr(K, "flash_set_dkdv2"):
    K.flash_set_dkdv2(False)
    tb = t(lambda: K.flash_bwd(do, qk, qkv, o, lse, S, Hq, Hkv, D, 1))
    print(f"{'bwd deterministic, 1-slice dK/dV':34s} {tb:7.1f} us  {5 * unit / tb / 1e6:6.0f} TF/s (5-matmul count)")
    K.flash_set_dkdv2(True)
if hasattr(K, "flash_set_dq_split"):  # dQ key split forced off / on (default: auto)
    for v in (0, 1):
        K.flash_set_dq_split(v)
        tb = t(lambda: K.flash_bwd(do, qk, qkv, o, lse, S, Hq, Hkv, D, 1))
        print(f"bwd deterministic, dQ split {'on ' if v else 'off'} {tb:7.1f} us  {5 * unit / tb / 1e6:6.0f} TF/s")
    K.flash_set_dq_split(-1)
if hasattr(K, "flash_set_kv_split"):  # dK/dV split forced off / on (default: auto, d=64)
    for v in (0, 1):
        K.flash_set_kv_split(v)
        tb = t(lambda: K.flash_bwd(do, qk, qkv, o, lse, S, Hq, Hkv, D, 1))
        print(f"bwd deterministic, dK/dV split {'on ' if v else 'off'} {tb:7.1f} us  {5 * unit / tb / 1e6:6.0f} TF/s")
    K.flash_set_kv_split(-1)
