"""Diagnoses a wrong w4 GEMM: fits the output, per 64 x 64 block, as a combination of the per-K-tile
partial products (out ~= sum_t c_t A[:, t] B[:, t]^T); a correct kernel gives c = 1 for every
K-tile, a stage / schedule bug shows up as the pattern of wrong coefficients.

    python scripts/w4_diag.py --nj 4 --m 512 --k 256 [--layout nt|dx|dw]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fault_tolerant_llm_training_amd._native import kernels  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nj", type=int, default=4)
    ap.add_argument("--m", type=int, default=512)
    ap.add_argument("--k", type=int, default=256)
    ap.add_argument("--layout", default="nt")
    args = ap.parse_args()
    K_ = kernels()
    torch.manual_seed(0)
    M, Kd, nj = args.m, args.k, args.nj
    N = 32 * nj * 3
    a = (torch.rand(M, Kd, device="cuda") * 2 - 1).bfloat16()
    b = (torch.rand(N, Kd, device="cuda") * 2 - 1).bfloat16()
    if args.layout == "nt":
        out = K_.gemm_nt_w4(a, b, None, None, nj)
    elif args.layout == "dx":
        out = K_.gemm_w4_ex(a, False, b.t().contiguous(), True, M, N, Kd, None, False, None, nj)
    else:
        out = K_.gemm_w4_ex(a.t().contiguous(), True, b.t().contiguous(), True, M, N, Kd, None, False,
                            None, nj)
    torch.cuda.synchronize()
    nk = Kd // 64
    parts = torch.stack([a[:, t * 64:(t + 1) * 64].float() @ b[:, t * 64:(t + 1) * 64].float().t()
                         for t in range(nk)])  # [nk, M, N]
    ref = parts.sum(0)
    print(f"nj={nj} M={M} N={N} K={Kd} layout={args.layout}: rel err "
          f"{((out.float() - ref).norm() / ref.norm()).item():.4f}")
    bad = 0
    for bm in range(0, M, 64):
        for bn in range(0, N, 64):
            o = out[bm:bm + 64, bn:bn + 64].float().reshape(-1)
            P = parts[:, bm:bm + 64, bn:bn + 64].reshape(nk, -1).t()
            c = torch.linalg.lstsq(P.cpu(), o.cpu()[:, None]).solution.reshape(-1)
            res = ((P.cpu() @ c - o.cpu()).norm() / o.cpu().norm()).item()
            if (c - 1).abs().max() > 0.02 or res > 0.02:
                bad += 1
                if bad <= 24:
                    print(f"  block m{bm:5d} n{bn:5d}: coeffs {[round(x, 2) for x in c.tolist()]} "
                          f"residual {res:.3f}")
    print(f"{bad} bad 64x64 blocks of {(M // 64) * (N // 64)}")


if __name__ == "__main__":
    main()
