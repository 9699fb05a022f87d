#!/usr/bin/env python3
"""HBM use of the 8B step by phase and step (allocated / reserved / per-step peak, GiB)."""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fault_tolerant_llm_training_amd.models.llama import build_model, model_args_for  # noqa: E402
from fault_tolerant_llm_training_amd.optim.adamw import FlatAdamW  # noqa: E402
from fault_tolerant_llm_training_amd.parallel.ddp import GradReducer  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--seq-len", type=int, default=2048)
ap.add_argument("--recompute", type=int, default=0)
ap.add_argument("--steps", type=int, default=4)
ap.add_argument("--model", default="llama3-8b")
ap.add_argument("--free-run", action="store_true", help="no host sync between steps (like bench.py)")
ap.add_argument("--throttle", action="store_true", help="with --free-run: at most one step in flight")
a = ap.parse_args()
G = 2**30


def mem(tag):
    torch.cuda.synchronize()
    print(f"{tag:28s} alloc {torch.cuda.memory_allocated() / G:7.1f}  reserved {torch.cuda.memory_reserved() / G:7.1f}"
          f"  peak {torch.cuda.max_memory_allocated() / G:7.1f}", flush=True)


dev = torch.device("cuda")
margs = model_args_for(a.model, vocab_size=131072, seq_len=a.seq_len)
m = build_model(margs, dev, torch.bfloat16)
mem("model")
m.set_activation_checkpointing(a.recompute)
red = GradReducer(m.flat, m.sinks_in_backward_order(), bucket_mb=256)
opt = FlatAdamW(m.parameters(), m.flat, lr=5e-5, max_grad_norm=1.0, reducer=red)
m.gate = opt.gate
mem("optimizer")
inv = torch.full((1,), 1.0 / a.seq_len, device=dev)
if a.free_run:
    prev = None
    for i in range(a.steps):
        tok = torch.randint(0, 131072, (1, a.seq_len), device=dev)
        lab = torch.randint(0, 131072, (1, a.seq_len), device=dev)
        loss = m(tok, lab, inv)
        loss.backward()
        red.finish()
        opt.step()
        ev = torch.cuda.Event()
        ev.record()
        if a.throttle and prev is not None:
            prev.synchronize()
        prev = ev
    st = torch.cuda.memory_stats()
    print(f"free-run{' throttled' if a.throttle else ''}: peak alloc {st['allocated_bytes.all.peak'] / G:.1f} "
          f"peak reserved {st['reserved_bytes.all.peak'] / G:.1f} retries {st['num_alloc_retries']}", flush=True)
    mem("end")
for i in range(0 if a.free_run else a.steps):
    torch.cuda.reset_peak_memory_stats()
    tok = torch.randint(0, 131072, (1, a.seq_len), device=dev)
    lab = torch.randint(0, 131072, (1, a.seq_len), device=dev)
    loss = m(tok, lab, inv)
    mem(f"step {i} after forward")
    loss.backward()
    mem(f"step {i} after backward")
    red.finish()
    opt.step()
    opt.gate.wait_all()
    mem(f"step {i} after optimizer")
    del loss
    mem(f"step {i} after del loss")
print(torch.cuda.memory_summary(abbreviated=True), flush=True)
