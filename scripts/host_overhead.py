"""Host enqueue time vs GPU time of one training step (is a preset launch-bound?), MI355X.

    python scripts/host_overhead.py [model]
For each of 10 steps: synchronize, then time the host call that enqueues the whole step
(forward, backward with its bucket hooks, optimizer) and, separately, the GPU time of the
step from events. host >= gpu means the GPU waits for the host."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fault_tolerant_llm_training_amd.data.synthetic import SyntheticTokens  # noqa: E402
from fault_tolerant_llm_training_amd.models.llama import build_model, model_args_for  # noqa: E402
from fault_tolerant_llm_training_amd.optim.adamw import FlatAdamW  # noqa: E402
from fault_tolerant_llm_training_amd.parallel.ddp import GradReducer  # noqa: E402

preset = sys.argv[1] if len(sys.argv) > 1 else "gpt2-small"
V, S = 131072, 2048
a = model_args_for(preset, vocab_size=V, seq_len=S)
m = build_model(a, "cuda", torch.bfloat16, seed=1)
red = GradReducer(m.flat, m.sinks_in_backward_order(), bucket_mb=256.0)
opt = FlatAdamW(m.parameters(), m.flat, lr=1e-4, max_grad_norm=1.0, reducer=red)
m.gate = opt.gate
data = SyntheticTokens(V, S, seed=3)
inv = torch.full((1,), 1.0 / S, device="cuda")


def step(i):
    x, y = data.batch(i, 1)
    loss = m(x.cuda(non_blocking=True), y.cuda(non_blocking=True), inv)
    loss.backward()
    red.finish()
    opt.step()


for i in range(5):
    step(i)
torch.cuda.synchronize()
hs, gs = [], []
for i in range(10):
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    t = time.perf_counter()
    step(5 + i)
    hs.append((time.perf_counter() - t) * 1e3)
    opt.gate.wait_all()
    e1.record()
    torch.cuda.synchronize()
    gs.append(e0.elapsed_time(e1))
hs.sort()
gs.sort()
print(f"{preset}: host enqueue {hs[5]:.2f} ms (median; min {hs[0]:.2f}), GPU step {gs[5]:.2f} ms (median; min {gs[0]:.2f})")
