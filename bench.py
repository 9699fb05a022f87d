#!/usr/bin/env python3
"""Headline benchmark: training tokens/s at seq-len 2048, data parallel over N MI355X.

Config (BASELINE.json / BASELINE.md): Llama-3-8B-shaped decoder (reference
train.py:43-53; vocab 131072 like the reference's Mistral-Nemo tokenizer),
seq 2048, batch 1 per GPU, bf16 params/grads/AdamW states, lr 5e-5 with 100
warmup steps, grad clipping at 1.0 — the reference's logged run (train.sh:16-20).
Synthetic tokens, random-init weights (no network on the GPU box). Every timed
step is a full training step: H2D of the batch, forward, backward with the
gradient buckets' RCCL collectives launched as backward produces them (ZeRO-1
reduce-scatter by default for N > 1; ``--dp-mode allreduce`` for replicated
state), gradient norm + clip, AdamW (+ parameter all-gather under ZeRO-1),
LR-scheduler step.

    python bench.py --gpus N --steps K --warmup W       (N > 1: starts N ranks itself, see self_launch)
    torchrun --nproc-per-node N bench.py --gpus N ...   (one rank per GPU)

The process group's size must equal ``--gpus`` (exit 2 otherwise), so an N-GPU row is always an
N-rank measurement.

Rank 0 prints one JSON line; ``value`` is the whole-job tokens/s (sum over
GPUs, the driver's contract), timed between barriers + device syncs, max step
time over ranks. ``vs_baseline`` compares like with like: tokens/s *per GPU*
against the reference's 6,376 tokens/s on its one GPU (the BASELINE metric is
"tokens/sec/GPU"), so it does not grow with N by itself.

After the timed steps (outside the timed region) the second half of the
BASELINE metric is measured on the same state: the checkpoint save wall-clock
(exit path, blocking until durable) and the training-visible cost of a
periodic save that overlaps the next steps (``ckpt_save``; ``--no-ckpt`` skips
it). Under data parallelism the collective exposure is estimated by re-running
the same steps with every collective skipped (``exposed_comm_ms_per_step``).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

BASELINE_TOK_S_PER_GPU = 6376.0  # 1x GH200, Llama-3-8B, seq 2048, bs 1
METRIC = "tokens/sec/GPU seq-len 2048 DP at 1/2/4/8 MI355X; checkpoint save wall-clock (s)"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--seq-len", type=int, default=2048)
    ap.add_argument("--batch-size", type=int, default=1)
    ap.add_argument("--vocab-size", type=int, default=131072)
    ap.add_argument("--bucket-mb", type=float, default=None,
                    help="gradient / optimizer bucket MiB (default: 64 on one GPU, 256 under DP)")
    ap.add_argument("--ckpt-dir", default="", help="directory for the checkpoint-save measurement "
                    "(default: $FT_BENCH_CKPT_DIR or <tmpdir>/ft_bench_ckpt)")
    ap.add_argument("--no-ckpt", action="store_true", help="skip the checkpoint-save measurement")
    ap.add_argument("--ckpt-mode", default="auto", choices=["auto", "hbm", "host"],
                    help="checkpoint snapshot: 'hbm' (D2D into spare HBM, then drained to host), 'host' "
                         "(straight to pinned host memory), 'auto' (hbm when the free HBM holds it)")
    ap.add_argument("--grad-accum", type=int, default=1, help="micro-batches per optimizer step")
    ap.add_argument("--no-exposed-comm", action="store_true", help="skip the DP exposed-collective estimate")
    ap.add_argument("--graph", action="store_true",
                    help="replay each step as one HIP graph (optimizer of step k with forward/backward of "
                         "step k+1, the RCCL bucket collectives captured under DP): launch-bound presets")
    ap.add_argument("--device", default="cuda")
    ap.add_argument("--dp-mode", default="", choices=["", "allreduce", "zero1"])
    ap.add_argument("--dp-reduce-dtype", default="native", choices=["native", "bf16", "fp32"],
                    help="gradient collectives in the model dtype (default) or on an fp32 copy")
    ap.add_argument("--no-overlap", action="store_true", help="per-bucket optimizer as a serial phase (A/B)")
    ap.add_argument("--activation-checkpointing", type=int, default=0,
                    help="recompute this many blocks in backward (-1 = all): long-context runs")
    ap.add_argument("--recompute-attention", action="store_true",
                    help="with --activation-checkpointing: re-run flash fwd too (default keeps its output)")
    ap.add_argument("--whole-buffer-optimizer", action="store_true",
                    help="1 GPU: one norm + one AdamW launch over the flat buffer after backward (A/B)")
    return ap.parse_args()


def _sync(dev):
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)


def _launched_world():
    """WORLD_SIZE of the launcher this process runs under (torchrun or Slurm), or None."""
    env = os.environ
    if "WORLD_SIZE" in env:
        return int(env["WORLD_SIZE"])
    if "SLURM_NTASKS" in env and "SLURM_PROCID" in env:
        return int(env["SLURM_NTASKS"])
    return None


def _free_port() -> int:
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def self_launch(a) -> int | None:
    """``--gpus N`` (N > 1) with no launcher: start N ranks as a child torchrun and return its exit
    code, so the N-GPU row can never be a 1-rank number. Runs before anything touches the GPU
    (``torch.cuda.device_count`` does not initialise HIP on this image); the child is a separate
    process, never an exec. Returns None when this process is already one rank of a launch."""
    world = _launched_world()
    if world is not None or a.gpus <= 1:
        return None
    if a.device == "cuda":
        have = torch.cuda.device_count()
        if have < a.gpus:
            print(f"[bench] --gpus {a.gpus} but only {have} GPU(s) visible", file=sys.stderr)
            return 2
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(a.gpus),
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__)] + sys.argv[1:]
    print(f"[bench] no launcher: starting {a.gpus} ranks ({' '.join(cmd[1:6])} ...)", file=sys.stderr, flush=True)
    import subprocess

    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


def main():
    a = parse()
    rc = self_launch(a)
    if rc is not None:
        sys.exit(rc)
    launched = _launched_world()
    if launched is not None and launched != a.gpus:
        print(f"[bench] --gpus {a.gpus} but the launcher started {launched} rank(s)", file=sys.stderr)
        sys.exit(2)
    from fault_tolerant_llm_training_amd.parallel import dist as fdist
    from fault_tolerant_llm_training_amd.parallel.ddp import GradReducer
    from fault_tolerant_llm_training_amd.models.llama import build_model, model_args_for, flops_per_token
    from fault_tolerant_llm_training_amd.optim.adamw import FlatAdamW
    from fault_tolerant_llm_training_amd.utils.lr import build_lr_scheduler
    from fault_tolerant_llm_training_amd.data.synthetic import SyntheticTokens

    # 5-minute collective timeout: a rank that fails inside the checkpoint block makes its peers
    # raise (and report the error in the JSON line) instead of blocking for the 30-minute default
    if a.graph:
        fdist.graph_capture_env()
    info = fdist.init_distributed(a.device, timeout_s=300)
    dev = info.device
    world = info.world_size
    # what the job really runs on: process-group size (must be --gpus), one distinct GPU per rank
    # (raises otherwise), peer access between every pair, RCCL version -- recorded in the JSON line
    topo = fdist.topology_report(info, expected_world=a.gpus)

    margs = model_args_for(a.model, vocab_size=a.vocab_size, seq_len=a.seq_len)
    model = build_model(margs, dev, torch.bfloat16, seed=1234)
    if a.activation_checkpointing:
        model.set_activation_checkpointing(a.activation_checkpointing, recompute_attention=a.recompute_attention)
    red = GradReducer(model.flat, model.sinks_in_backward_order(), bucket_mb=a.bucket_mb,
                      mode=a.dp_mode or None, overlap=not a.no_overlap, reduce_dtype=a.dp_reduce_dtype)
    if a.whole_buffer_optimizer and world == 1:
        for snk in list(model.flat.sinks.values()) + model.sinks_in_backward_order():
            snk.hook = None
        red.finish = lambda: None
    opt = FlatAdamW(model.parameters(), model.flat, lr=5e-5, max_grad_norm=1.0,
                    reducer=None if (a.whole_buffer_optimizer and world == 1) else red)
    model.gate = opt.gate
    sched = build_lr_scheduler(opt, 100)
    red.broadcast_params()

    data = SyntheticTokens(a.vocab_size, a.seq_len, seed=4321, rank=info.rank, world_size=world)
    B, S, K = a.batch_size, a.seq_len, max(1, a.grad_accum)
    inv_count = torch.full((1,), 1.0 / (B * K * S * world), dtype=torch.float32, device=dev)

    def step(i, before_opt=None):
        tok_all, lab_all = data.batch(i, B * K)
        tok_all = tok_all.to(dev, non_blocking=True)
        lab_all = lab_all.to(dev, non_blocking=True)
        loss = None
        for k in range(K):
            red.begin_micro(k, K)
            lk = model(tok_all[k * B:(k + 1) * B], lab_all[k * B:(k + 1) * B], inv_count)
            lk.backward()
            loss = lk.detach() if loss is None else loss + lk.detach()
        red.finish()
        opt.clip_grad_norm_(1.0)
        if before_opt is not None:
            before_opt()
        opt.step()
        sched.step()
        return loss

    graphed = None
    if a.graph:
        if K > 1 or dev.type != "cuda":
            raise SystemExit("--graph: GPU ranks, no gradient accumulation")
        from fault_tolerant_llm_training_amd.graphs import GraphedStep, hw_queue_problem

        if hw_queue_problem():
            raise SystemExit("--graph: " + hw_queue_problem())

        def fwd_bwd(tok, lab):
            loss_ = model(tok, lab, inv_count)
            loss_.backward()
            red.finish()
            return loss_

        graphed = GraphedStep(model, red, opt, sched, fwd_bwd)
    for i in range(a.warmup):
        if graphed is not None and i == a.warmup - 1:
            loss = graphed.prime(*data.batch(i, B))  # eager fwd/bwd of step i, then capture
        else:
            loss = step(i)
    sampler = None
    if dev.type == "cuda":
        from fault_tolerant_llm_training_amd.utils.telemetry import start_sampler

        sampler = start_sampler(dev.index or 0)
    _sync(dev)
    fdist.barrier()
    _sync(dev)
    if sampler is not None:
        sampler.on = True
    t0 = time.perf_counter()
    for i in range(a.steps):
        if graphed is not None:  # optimizer of step i-1 + forward/backward of step i
            loss = graphed.step(*data.batch(a.warmup + i, B))
        else:
            loss = step(a.warmup + i)
    opt.gate.wait_all()
    _sync(dev)
    fdist.barrier()
    _sync(dev)
    elapsed = time.perf_counter() - t0
    if sampler is not None:
        sampler.on = False
        sampler.stop_ = True
    if graphed is not None:
        graphed.finish()  # the last backward's optimizer step (outside the timed window)
        opt.graph_mode = False
    elapsed = fdist.ctrl_allreduce_max(int(elapsed * 1e9)) / 1e9
    # each rank's loss is its token sum over the GLOBAL token count: the global mean is the sum
    final_loss = fdist.ctrl_allreduce_sum(float(loss.item())) if world > 1 else float(loss.item())
    opt.check_finite(block=True)

    ms = elapsed / a.steps * 1e3
    tok_s = B * K * S * world * a.steps / elapsed
    fpt = flops_per_token(margs, S)
    mfu = tok_s / world * fpt / 2.5e15
    out = {
        "metric": METRIC,
        "value": round(tok_s, 1),
        "unit": "tokens/s (whole job, sum over GPUs)",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(ms, 2),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": round(tok_s / world / BASELINE_TOK_S_PER_GPU, 3),
        "vs_baseline_basis": "tokens/s per GPU / 6376 (reference, 1x GH200, BASELINE.md)",
        "dtype": "bf16",
        "data": "synthetic",
        "config": {"model": a.model, "global_batch": B * K * world, "seq_len": S, "parallelism": f"dp{world}"},
        # the metric is named per GPU; `value` is the driver's whole-job aggregate: both explicit
        "value_basis": "whole job: tokens/s summed over all n_gpus (per GPU: tokens_per_s_per_gpu)",
        "tokens_per_s_whole_job": round(tok_s, 1),
        "tokens_per_s_per_gpu": round(tok_s / world, 1),
        "mfu_vs_2.5PF_dense": round(mfu, 4),
        "final_loss": round(final_loss, 4),
        "params": model.num_params(),
        "grad_mode": red.mode,
        "buckets": len(red.buckets),
        # bytes each rank sends (and receives) per step in the gradient/parameter collectives:
        # reduce-scatter + all-gather (ZeRO-1) or all-reduce, 2(W-1)/W of the dense gradient
        "comm_GB_per_rank_per_step": round(
            2.0 * (world - 1) / world * sum(b.numel for b in red.buckets if not b.sparse)
            * model.flat.grads.element_size() / 1e9, 2),
        # sparse embedding exchange: each rank sends its B*S (token, dY row) pairs and receives
        # the other W-1 ranks' (all-gather)
        "sparse_emb_GB_received_per_rank_per_step": round(
            (world - 1) * B * K * S * (margs.dim * model.flat.grads.element_size() + 8) / 1e9, 3)
        if red.sparse_embedding else 0.0,
        "recompute_layers": model.recompute_layers,
        "world_size": topo["world_size"],
        "distinct_devices": topo["distinct_devices"],
        "device_ids": [d["id"] for d in topo["devices"]],
        "peer_access_all_pairs": topo["peer_access_all_pairs"],
        "rccl_version": topo["rccl_version"],
    }
    if sampler is not None:
        # board power / shader clock over the timed region (rank 0's GPU): they tell a hotter or
        # lower-clocked box from slower code. (No clock-normalised step time: across boxes the step
        # moved 0.55-0.65 % per 1 % of sclk, not 1:1 -- AdamW and the epilogues are memory-bound --
        # docs/PERFORMANCE.md "Clock and step time"; compare code on one box: scripts/ab_step.py.)
        out.update(sampler.summary())
    if a.dp_reduce_dtype == "fp32":
        out["dp_reduce_dtype"] = "fp32"
    if graphed is not None:
        out["hip_graph"] = True
    if dev.type == "cuda":
        ms_ = torch.cuda.memory_stats(dev)
        out["hbm_peak_gb"] = round(ms_.get("reserved_bytes.all.peak", 0) / 2**30, 1)
        out["alloc_retries"] = ms_.get("num_alloc_retries", 0)
    if K > 1:
        out["grad_accum"] = K
    nxt = a.warmup + a.steps
    if world > 1 and not a.no_exposed_comm:
        # same steps with every collective skipped: the difference is what the ranks wait for
        n = max(3, min(10, a.steps))
        red.dry_comm = True
        step(nxt)
        _sync(dev)
        t0 = time.perf_counter()
        for j in range(n):
            step(nxt + 1 + j)
        opt.gate.wait_all()
        _sync(dev)
        dry = (time.perf_counter() - t0) / n * 1e3
        red.dry_comm = False
        nxt += n + 1
        dry = fdist.ctrl_allreduce_max(int(dry * 1e6)) / 1e6
        out["compute_only_ms_per_step"] = round(dry, 2)
        out["exposed_comm_ms_per_step"] = round(ms - dry, 2)
    if not a.no_ckpt:
        import tempfile

        from fault_tolerant_llm_training_amd.ckpt.bench_save import measure_checkpoint

        d = a.ckpt_dir or os.environ.get("FT_BENCH_CKPT_DIR") or os.path.join(tempfile.gettempdir(), "ft_bench_ckpt")
        try:
            out["ckpt_save"] = measure_checkpoint(model, opt, sched, step, nxt, d, info, mode=a.ckpt_mode)
        except Exception as e:  # noqa: BLE001 - keep the throughput line; report why the save failed
            out["ckpt_save"] = {"error": repr(e)[:300], "dir": d}
    if info.is_main:
        print(json.dumps(out), flush=True)
    fdist.destroy()


if __name__ == "__main__":
    main()
