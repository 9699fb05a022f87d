#!/usr/bin/env python3
"""Same-process A/B of step-level knobs on the Llama-3-8B bench step (MI355X).

Knobs toggled between timing windows (alternating rounds, so box and clock drift cancel):
  hand_dw — weight-gradient GEMMs on the hand-written gfx950 kernel (row-major operands, no
          transposes) instead of hipBLASLt
  hand_dx — the dX GEMMs on the hand-written kernel
  hand_dw_wo_w2 / hand_dw_wo — only those weight gradients on the hand-written kernel
  dw    — weight-gradient GEMMs on a side stream, concurrent with the dX GEMMs
  sumsq_end — gradient-norm partial sums in one pass after backward instead of during it
  prio  — compute on a high-priority stream (its workgroups dispatch ahead of the side streams')
  dkdv2 — deterministic flash backward: slice-pair dK/dV kernel vs the one-slice kernel
  tonly — SwiGLU kernels write only the transposed activation/gradient; the w2 forward and
          w13 dX GEMMs read them as A^T
  qkvrope — QKV projection on the 4-wave hand GEMM with RoPE in its epilogue (no RoPE kernel)
  w4fwd — forward x W^T GEMMs with narrow tiles on the 4-wave hand GEMM (csrc/kernels/gemm_w4.hip)
  w4dw  — weight gradients on the 4-wave hand GEMM (transposed operands)
  notrans — weight gradients on hipBLASLt from the row-major operands (no transpose kernels)
  fastmath — AdamW / SwiGLU with the hardware v_rcp_f32 / v_sqrt_f32 instead of IEEE division/sqrt
  w4wide — the wide forward products (w13 at 224, the LM head at 256 columns) on the w4 GEMM too
  w4swiglu — the w1|w3 GEMM on the w4 kernel with SwiGLU in its epilogue (no separate SwiGLU pass)
  w4bwd — every dX / dW (and the FFN backward with the SwiGLU-backward epilogue) on the w4 kernel's
          k-major layouts (round 4) instead of hipBLASLt + transposed copies
  psums — the gradient-norm partials written by the dW / norm epilogues instead of a sumsq pass
  w4head — the LM-head logits GEMM on the w4 kernel
  r4    — w4bwd + psums + w4head together (round-4 routing vs round-3)
  deepdx — the deep-reduction dX products (8B w13 dX, LM-head dX) on hipBLASLt instead of the w4 kernel
  w4dwside — the w4 weight gradients on the dW side stream (default: inline on the compute stream)
  deadzero — the w4 GEMM's last two K-tiles issue their (dead) LDS-DMAs through null descriptors
          instead of re-staging the last K-tile (round 6)
  remainder — a 1.5-round dW grid (the 8B qkv dW) as a full round of 256-wide tiles plus the
          remaining rows at the 128-wide tile (round 6)
  cumask — the optimizer side stream (norm + AdamW) confined to every 4th CU (hipExtStreamCreateWithCUMask)
  cumask2 — ... to every 2nd CU
  f32mfma — (--dtype fp32) the fp32 model's GEMMs on the fp32 MFMA kernel instead of hipBLASLt
Usage: python scripts/ab_step.py [--steps 8] [--rounds 3] [--configs gemm,dw ...]
"""
from __future__ import annotations

import argparse
import itertools
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--seq-len", type=int, default=2048)
    ap.add_argument("--vocab-size", type=int, default=131072)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--steps", type=int, default=8)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--knobs", default="splitk")
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp16", "fp32"])
    a = ap.parse_args()

    from fault_tolerant_llm_training_amd.data.synthetic import SyntheticTokens
    from fault_tolerant_llm_training_amd.models.llama import build_model, model_args_for
    from fault_tolerant_llm_training_amd.ops import functional as Fx
    from fault_tolerant_llm_training_amd.optim.adamw import FlatAdamW
    from fault_tolerant_llm_training_amd.parallel.ddp import GradReducer
    from fault_tolerant_llm_training_amd.utils.lr import build_lr_scheduler

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    margs = model_args_for(a.model, vocab_size=a.vocab_size, seq_len=a.seq_len)
    dt = {"bf16": torch.bfloat16, "fp16": torch.float16, "fp32": torch.float32}[a.dtype]
    model = build_model(margs, dev, dt, seed=1234)
    red = GradReducer(model.flat, model.sinks_in_backward_order())  # bench.py's default buckets
    opt = FlatAdamW(model.parameters(), model.flat, lr=5e-5, max_grad_norm=1.0, reducer=red)
    model.gate = opt.gate
    sched = build_lr_scheduler(opt, 100)
    data = SyntheticTokens(a.vocab_size, a.seq_len, seed=4321)
    inv = torch.full((1,), 1.0 / a.seq_len, dtype=torch.float32, device=dev)
    it = [0]
    serial_adamw = [False]

    def step():
        tok, lab = data.batch(it[0], 1)
        it[0] += 1
        loss = model(tok.to(dev, non_blocking=True), lab.to(dev, non_blocking=True), inv)
        loss.backward()
        red.finish()
        opt.clip_grad_norm_(1.0)
        opt.step()
        if serial_adamw[0]:  # the next forward starts after the whole optimizer step
            opt.gate.wait_all()
        sched.step()
        return loss

    def window(n):
        opt.gate.wait_all()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(n):
            step()
        opt.gate.wait_all()
        torch.cuda.synchronize()
        return (time.perf_counter() - t) / n * 1e3

    knobs = [k for k in a.knobs.split(",") if k]
    from fault_tolerant_llm_training_amd._native import kernels
    from fault_tolerant_llm_training_amd.parallel import ddp as ddp_mod

    hp = torch.cuda.Stream(device=dev, priority=-1)
    default_stream = torch.cuda.current_stream(dev)

    def set_prio(on):
        torch.cuda.synchronize()
        torch.cuda.set_stream(hp if on else default_stream)

    setters = {"dw": Fx.set_dw_stream, "dkdv2": kernels().flash_set_dkdv2, "prio": set_prio,
               "sumsq_end": ddp_mod.set_sumsq_at_end, "qkvrope": Fx.set_qkv_rope, "w4fwd": Fx.set_w4_fwd,
               "fastmath": lambda on: (torch.cuda.synchronize(), kernels().set_exact_math(not on)),
               "w4swiglu": lambda on: (torch.cuda.synchronize(), Fx.set_w4_swiglu(on)),
               "w4bwd": lambda on: (torch.cuda.synchronize(), Fx.set_w4_bwd(on)),
               "psums": lambda on: (torch.cuda.synchronize(), red.set_producer_sums(on)),
               "splitk": lambda on: (torch.cuda.synchronize(), Fx.set_w4_splitk(1 if on else 0)),
               "w4dwside": lambda on: (torch.cuda.synchronize(), setattr(Fx, "_W4_DW_SIDE", on)),
               "gemm_s": lambda on: (torch.cuda.synchronize(), Fx.set_gemm_s(on)),
               "adamw_serial": lambda on: serial_adamw.__setitem__(0, bool(on)),
               "raster": lambda on: (torch.cuda.synchronize(), kernels().gemm_w4_set_group(-1 if on else 0)),
               "deadzero": lambda on: (torch.cuda.synchronize(), kernels().gemm_w4_set_deadzero(1 if on else 0)),
               "f32mfma": lambda on: (torch.cuda.synchronize(), Fx.set_f32_mfma(on)),
               "remainder": lambda on: (torch.cuda.synchronize(), kernels().gemm_w4_set_remainder(1 if on else 0))}
    side0 = red.side
    masked = {}

    def set_cumask(stride, on):
        torch.cuda.synchronize()
        if on and stride not in masked:
            masked[stride] = torch.cuda.ExternalStream(kernels().cu_masked_stream(stride, 0), device=dev)
        red.side = masked[stride] if on else side0

    setters["cumask"] = lambda on: set_cumask(4, on)
    setters["cumask2"] = lambda on: set_cumask(2, on)
    configs = list(itertools.product([False, True], repeat=len(knobs)))

    def apply(cfg):
        for k, on in zip(knobs, cfg):
            setters[k](on)

    for cfg in configs:  # warm every configuration (allocator pools, side streams)
        apply(cfg)
        for _ in range(a.warmup):
            step()
    res = {cfg: [] for cfg in configs}
    for r in range(a.rounds):
        for cfg in configs:
            apply(cfg)
            ms = window(a.steps)
            res[cfg].append(ms)
            name = " ".join(f"{k}={'on' if on else 'off'}" for k, on in zip(knobs, cfg))
            print(f"[ab] round {r} {name}: {ms:.2f} ms/step", flush=True)
    base = min(res[configs[0]])
    for cfg in configs:
        name = " ".join(f"{k}={'on' if on else 'off'}" for k, on in zip(knobs, cfg))
        best = min(res[cfg])
        print(f"[ab] {name:24s} best {best:7.2f} ms/step  median {sorted(res[cfg])[len(res[cfg]) // 2]:7.2f}  "
              f"{base / best:.3f}x vs all-off  ({a.seq_len * 1000 / best:.0f} tok/s)", flush=True)
    loss = step()
    torch.cuda.synchronize()
    print(f"[ab] final loss {float(loss):.4f}", flush=True)


if __name__ == "__main__":
    main()
