"""Host time of each phase of the eager Llama-3-8B step (bench.py's step) vs the GPU time per step: is
the host ever behind the GPU (idle gaps at the end of backward in rocprof traces)?
    python scripts/host_step_probe.py [steps]
"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fault_tolerant_llm_training_amd.data.synthetic import SyntheticTokens  # noqa: E402
from fault_tolerant_llm_training_amd.models.llama import build_model, model_args_for  # noqa: E402
from fault_tolerant_llm_training_amd.optim.adamw import FlatAdamW  # noqa: E402
from fault_tolerant_llm_training_amd.parallel.ddp import GradReducer  # noqa: E402
from fault_tolerant_llm_training_amd.utils.lr import build_lr_scheduler  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 12
    V, S = 131072, 2048
    dev = torch.device("cuda", 0)
    a = model_args_for("llama3-8b", vocab_size=V, seq_len=S)
    model = build_model(a, dev, torch.bfloat16, seed=1234)
    red = GradReducer(model.flat, model.sinks_in_backward_order(), bucket_mb=256.0)
    opt = FlatAdamW(model.parameters(), model.flat, lr=5e-5, max_grad_norm=1.0, reducer=red)
    model.gate = opt.gate
    sched = build_lr_scheduler(opt, 100)
    data = SyntheticTokens(V, S, seed=4321)
    inv = torch.full((1,), 1.0 / S, dtype=torch.float32, device=dev)
    parts = {k: 0.0 for k in ("batch", "forward", "backward", "finish", "opt", "sched")}

    def step(i, acc):
        t = time.perf_counter()
        tok, lab = data.batch(i, 1)
        tok, lab = tok.to(dev, non_blocking=True), lab.to(dev, non_blocking=True)
        t1 = time.perf_counter()
        loss = model(tok, lab, inv)
        t2 = time.perf_counter()
        loss.backward()
        t3 = time.perf_counter()
        red.finish()
        t4 = time.perf_counter()
        opt.clip_grad_norm_(1.0)
        opt.step()
        t5 = time.perf_counter()
        sched.step()
        t6 = time.perf_counter()
        if acc:
            for k, dt in zip(parts, (t1 - t, t2 - t1, t3 - t2, t4 - t3, t5 - t4, t6 - t5)):
                parts[k] += dt

    for i in range(4):
        step(i, False)
    opt.gate.wait_all()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(n):
        step(4 + i, True)
    host = (time.perf_counter() - t0) / n * 1e3
    opt.gate.wait_all()
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / n * 1e3
    print(f"8B eager step: host {host:.2f} ms/step, wall {wall:.2f} ms/step | " +
          ", ".join(f"{k} {v / n * 1e3:.2f}" for k, v in parts.items()), flush=True)


if __name__ == "__main__":
    main()
