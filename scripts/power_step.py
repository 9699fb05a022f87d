"""Board power and shader clock during the real Llama-3-8B training step (bench.py's step: forward,
backward, grad norm, AdamW pipelined into the next forward) next to the isolated GEMM chain and
AdamW of scripts/power_probe.py — is the whole step at the board power limit, or only its phases?

    python scripts/power_step.py [seconds]
"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from power_probe import Sampler, hwmons, ours, summarize  # noqa: E402


def main():
    secs = float(sys.argv[1]) if len(sys.argv) > 1 else 4.0
    from fault_tolerant_llm_training_amd.data.synthetic import SyntheticTokens
    from fault_tolerant_llm_training_amd.models.llama import build_model, model_args_for
    from fault_tolerant_llm_training_amd.optim.adamw import FlatAdamW
    from fault_tolerant_llm_training_amd.parallel.ddp import GradReducer
    from fault_tolerant_llm_training_amd.utils.lr import build_lr_scheduler

    mons = hwmons()
    torch.cuda.init()
    mons = ours(mons)
    dev = torch.device("cuda", 0)
    V, S = 131072, 2048
    margs = model_args_for("llama3-8b", vocab_size=V, seq_len=S)
    model = build_model(margs, dev, torch.bfloat16, seed=1234)
    red = GradReducer(model.flat, model.sinks_in_backward_order(), bucket_mb=256.0)
    opt = FlatAdamW(model.parameters(), model.flat, lr=5e-5, max_grad_norm=1.0, reducer=red)
    model.gate = opt.gate
    sched = build_lr_scheduler(opt, 100)
    data = SyntheticTokens(V, S, seed=4321)
    inv = torch.full((1,), 1.0 / S, dtype=torch.float32, device=dev)

    def step(i):
        tok, lab = data.batch(i, 1)
        loss = model(tok.to(dev, non_blocking=True), lab.to(dev, non_blocking=True), inv)
        loss.backward()
        red.finish()
        opt.clip_grad_norm_(1.0)
        opt.step()
        sched.step()

    smp = Sampler(mons)
    smp.start()
    time.sleep(0.5)
    smp.on = True
    time.sleep(1.0)
    smp.on = False
    summarize("idle", list(smp.samples), mons, 0.0)
    for i in range(4):
        step(i)
    opt.gate.wait_all()
    torch.cuda.synchronize()
    smp.samples = []
    smp.on = True
    n, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < secs:
        step(4 + n)
        n += 1
    opt.gate.wait_all()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / n * 1e3
    smp.on = False
    summarize(f"8B training step ({n} steps)", list(smp.samples), mons, dt)
    # per-sample distribution: how much of the step sits at the limit
    pw = sorted(s[0].get("power1_average", s[0].get("power1_input", 0)) / 1e6 for s in smp.samples if s)
    sc = sorted(s[0].get("freq1_input", 0) / 1e6 for s in smp.samples if s)
    if pw:
        q = lambda xs, f: xs[min(len(xs) - 1, int(f * len(xs)))]
        print(f"power W  p10 {q(pw, .1):6.0f} p50 {q(pw, .5):6.0f} p90 {q(pw, .9):6.0f} | "
              f"sclk MHz p10 {q(sc, .1):6.0f} p50 {q(sc, .5):6.0f} p90 {q(sc, .9):6.0f} | {len(pw)} samples", flush=True)
    smp.stop_ = True


if __name__ == "__main__":
    main()
