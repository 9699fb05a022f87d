import torch, sys, os
sys.path.insert(0, os.getcwd())
from fault_tolerant_llm_training_amd._native import kernels
K = kernels()
r = lambda *s: (torch.rand(*s, device="cuda") * 2 - 1).bfloat16()
for (M, N, Kd) in [(6144, 4096, 2048), (4096, 4096, 2048), (4096, 14336, 2048)]:
    at, bt = r(Kd, M), r(Kd, N)
    for nj in (4, 7, 8):
        if N % (32 * nj): continue
        for _ in range(3): K.gemm_w4_ex(at, True, bt, True, M, N, Kd, None, False, None, nj)
        e = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        e[0].record()
        for _ in range(50): K.gemm_w4_ex(at, True, bt, True, M, N, Kd, None, False, None, nj)
        e[1].record(); torch.cuda.synchronize()
        us = e[0].elapsed_time(e[1]) / 50 * 1e3
        print(f"dW {M}x{N}x{Kd} nj={nj}: {us:.1f} us {2*M*N*Kd/us/1e6:.0f} TF/s (pick {K.gemm_w4_pick(M, N)})", flush=True)
