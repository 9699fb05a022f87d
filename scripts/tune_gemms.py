#!/usr/bin/env python3
"""Tune the GEMM solutions of one Llama-3-8B training step on an MI355X and A/B them.

1. builds the bench.py model/optimizer and runs warmup steps with the library heuristic;
2. enables PyTorch TunableOp tuning and runs ONE training step: every distinct GEMM the
   step issues (forward, dX, dW, at the layouts ops/functional.py uses) is benchmarked over
   all hipBLASLt and rocBLAS solutions and the fastest is kept;
3. times alternating windows heuristic / tuned in the same process (box and clock drift
   cancel out of the comparison);
4. TunableOp writes the table at exit (``--out``, default tuning/gemm_gfx950.csv).

A heartbeat line every 20 s keeps the GPU-box watchdog informed during tuning.
"""
from __future__ import annotations

import argparse
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ["FT_TUNED_GEMM"] = "0"  # this script drives TunableOp itself

import torch  # noqa: E402
import torch.cuda.tunable as tunable  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(ROOT, "tuning", "gemm_gfx950.csv"))
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--seq-len", type=int, default=2048)
    ap.add_argument("--vocab-size", type=int, default=131072)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--steps", type=int, default=8)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--tuning-ms", type=int, default=25, help="max time per candidate solution")
    ap.add_argument("--ab-only", action="store_true", help="load --out and only run the A/B")
    a = ap.parse_args()

    from fault_tolerant_llm_training_amd.data.synthetic import SyntheticTokens
    from fault_tolerant_llm_training_amd.models.llama import build_model, model_args_for
    from fault_tolerant_llm_training_amd.optim.adamw import FlatAdamW
    from fault_tolerant_llm_training_amd.parallel.ddp import GradReducer
    from fault_tolerant_llm_training_amd.utils.lr import build_lr_scheduler

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    tunable.set_filename(a.out, False)
    tunable.set_max_tuning_duration(a.tuning_ms)
    tunable.set_max_tuning_iterations(100)

    margs = model_args_for(a.model, vocab_size=a.vocab_size, seq_len=a.seq_len)
    model = build_model(margs, dev, torch.bfloat16, seed=1234)
    red = GradReducer(model.flat, model.sinks_in_backward_order(), bucket_mb=256.0)
    opt = FlatAdamW(model.parameters(), model.flat, lr=5e-5, max_grad_norm=1.0, reducer=red)
    model.gate = opt.gate
    sched = build_lr_scheduler(opt, 100)
    data = SyntheticTokens(a.vocab_size, a.seq_len, seed=4321)
    inv = torch.full((1,), 1.0 / a.seq_len, dtype=torch.float32, device=dev)
    it = [0]

    def step():
        tok, lab = data.batch(it[0], 1)
        it[0] += 1
        loss = model(tok.to(dev, non_blocking=True), lab.to(dev, non_blocking=True), inv)
        loss.backward()
        red.finish()
        opt.clip_grad_norm_(1.0)
        opt.step()
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

    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()
    print(f"[tune] heuristic warm: {window(a.steps):.2f} ms/step", flush=True)

    if a.ab_only:
        tunable.enable(True)
        tunable.tuning_enable(False)
        ok = tunable.read_file(a.out)
        print(f"[tune] loaded {a.out}: {ok}", flush=True)
    else:
        stop = threading.Event()
        t0 = time.time()

        def beat():
            while not stop.wait(20):
                print(f"[tune] tuning... {time.time() - t0:.0f}s, {len(tunable.get_results())} GEMMs done", flush=True)

        th = threading.Thread(target=beat, daemon=True)
        th.start()
        tunable.enable(True)
        tunable.tuning_enable(True)
        step()
        torch.cuda.synchronize()
        stop.set()
        th.join()
        print(f"[tune] tuned one step in {time.time() - t0:.0f}s", flush=True)
        for r in tunable.get_results():
            print("[tune] result", ",".join(str(x) for x in r), flush=True)
        # keep tuning enabled (nothing left to tune) so the table is written at exit

    for r in range(a.rounds):
        tunable.enable(False)
        d = window(a.steps)
        tunable.enable(True)
        t = window(a.steps)
        print(f"[tune] round {r}: heuristic {d:.2f} ms/step | tuned {t:.2f} ms/step | {d / t:.3f}x", flush=True)
    loss = step()
    torch.cuda.synchronize()
    print(f"[tune] final loss {float(loss):.4f}", flush=True)


if __name__ == "__main__":
    main()
