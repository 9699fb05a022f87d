"""Shader clock and board power per phase of the Llama-3-8B step (forward / backward / clip+AdamW),
to check how the step time should move with a box's clock (docs/PERFORMANCE.md "Box-to-box
variance").

The phases run serially here (a sync between them), so each one's samples are its own; bench.py's
step overlaps AdamW with the next forward, which this cannot separate. A background thread reads
the board's hwmon (power1_average, freq1_input) every 5 ms with a timestamp; each sample is
assigned to the phase whose [start, end) holds it.

    python scripts/phase_clock.py [steps]
"""
import os
import sys
import threading
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from fault_tolerant_llm_training_amd.utils.telemetry import _read_int, hwmon_for_pci_bus  # noqa: E402


class Stamped(threading.Thread):
    def __init__(self, hwmon, period_s=0.005):
        super().__init__(daemon=True)
        self.p = next((os.path.join(hwmon, n) for n in ("power1_average", "power1_input")
                       if os.path.exists(os.path.join(hwmon, n))), None)
        self.f = os.path.join(hwmon, "freq1_input")
        self.period_s, self.stop_, self.samples = period_s, False, []

    def run(self):
        while not self.stop_:
            t = time.perf_counter()
            pw, fq = _read_int(self.p), _read_int(self.f)
            if pw is not None and fq is not None:
                self.samples.append((t, pw / 1e6, fq / 1e6))
            time.sleep(self.period_s)


def q(xs, f):
    s = sorted(xs)
    return s[min(len(s) - 1, int(f * len(s)))] if s else float("nan")


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 30
    from fault_tolerant_llm_training_amd.data.synthetic import SyntheticTokens
    from fault_tolerant_llm_training_amd.models.llama import build_model, model_args_for
    from fault_tolerant_llm_training_amd.optim.adamw import FlatAdamW
    from fault_tolerant_llm_training_amd.parallel.ddp import GradReducer

    dev = torch.device("cuda", 0)
    hw = hwmon_for_pci_bus(getattr(torch.cuda.get_device_properties(0), "pci_bus_id", None))
    if hw is None:
        print("no hwmon for this board", flush=True)
        return
    V, S = 131072, 2048
    margs = model_args_for("llama3-8b", vocab_size=V, seq_len=S)
    model = build_model(margs, dev, torch.bfloat16, seed=1234)
    red = GradReducer(model.flat, model.sinks_in_backward_order(), bucket_mb=256.0)
    opt = FlatAdamW(model.parameters(), model.flat, lr=5e-5, max_grad_norm=1.0, reducer=red)
    model.gate = opt.gate
    data = SyntheticTokens(V, S, seed=4321)
    inv = torch.full((1,), 1.0 / S, dtype=torch.float32, device=dev)

    spans = {"forward": [], "backward": [], "clip+adamw": []}

    def step(i, record):
        tok, lab = data.batch(i, 1)
        tok, lab = tok.to(dev), lab.to(dev)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        loss = model(tok, lab, inv)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        loss.backward()
        red.finish()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        opt.clip_grad_norm_(1.0)
        opt.step()
        opt.gate.wait_all()
        torch.cuda.synchronize()
        t3 = time.perf_counter()
        if record:
            spans["forward"].append((t0, t1))
            spans["backward"].append((t1, t2))
            spans["clip+adamw"].append((t2, t3))

    for i in range(3):
        step(i, False)
    smp = Stamped(hw)
    smp.start()
    for i in range(steps):
        step(3 + i, True)
    smp.stop_ = True
    smp.join()
    print(f"Llama-3-8B, seq {S}, phases serialised, {steps} steps, {len(smp.samples)} hwmon samples "
          f"every ~5 ms (power1_average is the SMU's running average: it smears across phase edges)",
          flush=True)
    print(f"{'phase':12s} {'ms':>8s} {'sclk p10':>9s} {'p50':>6s} {'p90':>6s} {'power p50':>10s} {'n':>5s}")
    tot = {}
    for name, sp in spans.items():
        ms = sum(b - a for a, b in sp) / len(sp) * 1e3
        tot[name] = ms
        # drop the first 2 ms of each span: the hwmon power is an average over the previous phase
        ins = [(p, f) for (t, p, f) in smp.samples if any(a + 2e-3 <= t < b for a, b in sp)]
        sc = [f for _, f in ins]
        pw = [p for p, _ in ins]
        print(f"{name:12s} {ms:8.2f} {q(sc, .1):9.0f} {q(sc, .5):6.0f} {q(sc, .9):6.0f} "
              f"{q(pw, .5):10.0f} {len(ins):5d}", flush=True)
    print(f"serial step {sum(tot.values()):.2f} ms", flush=True)


if __name__ == "__main__":
    main()
