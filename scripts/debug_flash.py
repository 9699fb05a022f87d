import torch, sys
sys.path.insert(0, '.')
from fault_tolerant_llm_training_amd._native import kernels
from tests.test_flash_attn_gpu import ref_attn, rel
K = kernels()
for (B,S,Hq,Hkv,D) in [(1,32,1,1,128),(1,64,1,1,128),(1,128,1,1,128),(1,256,1,1,128),(1,128,2,1,128),(1,64,1,1,64),(1,256,2,2,64)]:
    torch.manual_seed(0)
    T=B*S
    qkv = torch.randn(T, (Hq + 2 * Hkv) * D, device="cuda").bfloat16()
    qk = torch.randn(T, (Hq + Hkv) * D, device="cuda").bfloat16()
    o, lse = K.flash_fwd(qk, qkv, S, Hq, Hkv, D)
    q = qk[:, : Hq * D].float().view(B, S, Hq, D).requires_grad_(True)
    k = qk[:, Hq * D :].float().view(B, S, Hkv, D).requires_grad_(True)
    v = qkv[:, (Hq + Hkv) * D :].float().view(B, S, Hkv, D).requires_grad_(True)
    ref = ref_attn(q, k, v)
    do = torch.randn(T, Hq * D, device="cuda").bfloat16()
    dqkv = K.flash_bwd(do, qk, qkv, o, lse, S, Hq, Hkv, D)
    gq, gk, gv = torch.autograd.grad(ref, (q, k, v), do.float().view(B, S, Hq, D))
    eq = rel(dqkv[:, : Hq * D].view(B, S, Hq, D), gq)
    ek = rel(dqkv[:, Hq * D : (Hq + Hkv) * D].view(B, S, Hkv, D), gk)
    ev = rel(dqkv[:, (Hq + Hkv) * D :].view(B, S, Hkv, D), gv)
    print(B,S,Hq,Hkv,D, 'o', round(rel(o.view(B,S,Hq,D), ref),4), 'dq', round(eq,4), 'dk', round(ek,4), 'dv', round(ev,4))
    if S <= 64 and D == 128:
        a = dqkv[:, :D].float(); b = gq.view(T, -1)[:, :D]
        print(' dq row1 ours', a[1,:6].tolist()); print(' dq row1 ref ', b[1,:6].tolist())
        print(' ratio rows', [(a[i].norm()/(b[i].norm()+1e-9)).item() for i in range(0, S, 7)])
