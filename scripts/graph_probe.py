"""Feasibility/perf probe: capture forward+backward (with the reducer's side-stream hooks) in a
HIP graph and replay it; optimizer stays eager. Compares step time vs eager."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fault_tolerant_llm_training_amd.models.llama import build_model, model_args_for  # noqa: E402
from fault_tolerant_llm_training_amd.optim.adamw import FlatAdamW  # noqa: E402
from fault_tolerant_llm_training_amd.parallel.ddp import GradReducer  # noqa: E402

preset = sys.argv[1] if len(sys.argv) > 1 else "gpt2-small"
V, S = 131072, 2048
a = model_args_for(preset, vocab_size=V, seq_len=S)


def setup():
    m = build_model(a, "cuda", torch.bfloat16, seed=1)
    red = GradReducer(m.flat, m.sinks_in_backward_order(), bucket_mb=256.0)
    opt = FlatAdamW(m.parameters(), m.flat, lr=1e-4, max_grad_norm=1.0, reducer=red)
    m.gate = opt.gate
    return m, red, opt


tok = torch.randint(0, V, (1, S), device="cuda")
lab = torch.randint(0, V, (1, S), device="cuda")
inv = torch.full((1,), 1.0 / S, device="cuda")


def timed(fn, n=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / n * 1e3


m, red, opt = setup()


def eager():
    loss = m(tok, lab, inv)
    loss.backward()
    red.finish()
    opt.step()
    return loss


print(f"{preset} eager: {timed(eager):.2f} ms/step", flush=True)

m, red, opt = setup()
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    for _ in range(3):  # warm up on the side stream (allocator pools, lazy init)
        eager()
torch.cuda.current_stream().wait_stream(s)
torch.cuda.synchronize()
opt.gate.wait_all()
g = torch.cuda.CUDAGraph()
m.gate = None  # the optimizer runs outside the graph; the replay waits for it as a whole
with torch.cuda.graph(g):
    loss_static = m(tok, lab, inv)
    loss_static.backward()
    red.finish()
    torch.cuda.current_stream().wait_stream(red.side)


def graphed():
    opt.gate.wait_all()
    g.replay()
    opt.step()


print(f"{preset} graph fwd+bwd: {timed(graphed):.2f} ms/step  loss={loss_static.item():.4f}", flush=True)
