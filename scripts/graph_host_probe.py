"""Is the GPT-2 whole-step HIP graph replay host-bound? Host time of each part of GraphedStep.step
(batch synthesis + pinning, hyper staging, batch H2D enqueue, graph.replay(), stats publish,
scheduler) for back-to-back steps, vs the GPU time per step.
    python scripts/graph_host_probe.py [model]
"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fault_tolerant_llm_training_amd.data.synthetic import SyntheticTokens  # noqa: E402
from fault_tolerant_llm_training_amd.graphs import GraphedStep  # noqa: E402
from fault_tolerant_llm_training_amd.models.llama import build_model, model_args_for  # noqa: E402
from fault_tolerant_llm_training_amd.optim.adamw import FlatAdamW  # noqa: E402
from fault_tolerant_llm_training_amd.parallel.ddp import GradReducer  # noqa: E402
from fault_tolerant_llm_training_amd.utils.lr import build_lr_scheduler  # noqa: E402


def main():
    preset = sys.argv[1] if len(sys.argv) > 1 else "gpt2-small"
    V, S = 131072, 2048
    dev = torch.device("cuda", 0)
    a = model_args_for(preset, vocab_size=V, seq_len=S)
    model = build_model(a, dev, torch.bfloat16, seed=1234)
    red = GradReducer(model.flat, model.sinks_in_backward_order(), bucket_mb=256.0)
    opt = FlatAdamW(model.parameters(), model.flat, lr=5e-5, max_grad_norm=1.0, reducer=red)
    model.gate = opt.gate
    sched = build_lr_scheduler(opt, 100)
    data = SyntheticTokens(V, S, seed=4321)
    inv = torch.full((1,), 1.0 / S, dtype=torch.float32, device=dev)

    def fwd_bwd(tok, lab):
        loss = model(tok, lab, inv)
        loss.backward()
        red.finish()
        return loss

    g = GraphedStep(model, red, opt, sched, fwd_bwd)
    for i in range(2):
        loss = fwd_bwd(*[t.to(dev) for t in data.batch(i, 1)])
        opt.clip_grad_norm_(1.0)
        opt.step()
        sched.step()
    g.prime(*data.batch(2, 1))
    for i in range(5):
        g.step(*data.batch(3 + i, 1))
    torch.cuda.synchronize()
    parts = {k: 0.0 for k in ("batch", "hyper", "h2d", "replay", "publish", "sched")}
    n = 40
    t_all = time.perf_counter()
    for i in range(n):
        t = time.perf_counter()
        tok, lab = data.batch(10 + i, 1)
        t1 = time.perf_counter(); parts["batch"] += t1 - t
        opt.step_count += 1
        opt.stage_hyper(opt.step_count)
        t2 = time.perf_counter(); parts["hyper"] += t2 - t1
        g.tok.copy_(tok, non_blocking=True)
        g.lab.copy_(lab, non_blocking=True)
        t3 = time.perf_counter(); parts["h2d"] += t3 - t2
        g.graph.replay()
        t4 = time.perf_counter(); parts["replay"] += t4 - t3
        opt.publish_stats()
        t5 = time.perf_counter(); parts["publish"] += t5 - t4
        sched.step()
        parts["sched"] += time.perf_counter() - t5
    host = (time.perf_counter() - t_all) / n * 1e3
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t_all) / n * 1e3
    print(f"{preset}: host enqueue {host:.2f} ms/step, wall {wall:.2f} ms/step | " +
          ", ".join(f"{k} {v / n * 1e3:.3f}" for k, v in parts.items()), flush=True)
    # GPU-only time of one replay (host ahead: replay several, time with events)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for i in range(10):
        g.graph.replay()
    e1.record()
    torch.cuda.synchronize()
    print(f"{preset}: 10 back-to-back replays (no host staging): {e0.elapsed_time(e1) / 10:.2f} ms/replay", flush=True)
    g.finish()


if __name__ == "__main__":
    main()
