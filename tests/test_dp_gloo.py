"""Data parallelism on the CPU with gloo (world_size 2): the RCCL code path's semantics.

* FlatDDP (bucketed all-reduce launched from backward, SUM of globally
  normalised losses) reproduces the single-process gradient of the global batch;
* ``train.py`` under torchrun: a SIGUSR1 delivered to ONE rank stops every
  rank at the same step (MAX vote), rank 0 writes the checkpoint, and the
  DP resume is bit-identical to an uninterrupted DP run.
"""
import os
import re
import signal
import socket
import subprocess
import sys
import time

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from helpers import ROOT, TINY, env_for, kill_group, wait_for_log, write_fake_sbatch

pytestmark = pytest.mark.slow


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out_dir, bucket_mb, mode):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from fault_tolerant_llm_training_amd.data.synthetic import SyntheticTokens
    from fault_tolerant_llm_training_amd.models.llama import build_model, model_args_for
    from fault_tolerant_llm_training_amd.parallel.ddp import GradReducer

    a = model_args_for("tiny", vocab_size=128, seq_len=16)
    m = build_model(a, "cpu", torch.float32, seed=5)
    ddp = GradReducer(m.flat, m.sinks_in_backward_order(), bucket_mb=bucket_mb, mode=mode)
    assert ddp.mode == mode
    ddp.broadcast_params()
    ds = SyntheticTokens(128, 16, seed=9, rank=rank, world_size=world, pin=False)
    for step in range(2):
        x, y = ds.batch(step, 2)
        y[0, :3] = -100  # uneven loss-token counts across ranks
        n = torch.tensor([float((y != -100).sum())])
        dist.all_reduce(n)
        loss = m(x, y, 1.0 / n)
        loss.backward()
        ddp.finish()
    if mode == "allreduce":
        assert any(b.sparse for b in ddp.buckets)  # the embedding is exchanged sparsely
        torch.save(m.flat.grads.clone(), os.path.join(out_dir, f"g{rank}.pt"))
    else:  # scatter this rank's reduced shards back into a full-layout tensor
        full = torch.full_like(m.flat.grads, float("nan"))
        for b in ddp.buckets:
            lo = b.lo + rank * b.shard_len
            full[lo : lo + b.shard_len] = ddp.grad_for_update(b)
        torch.save(full, os.path.join(out_dir, f"g{rank}.pt"))
    dist.destroy_process_group()


@pytest.mark.parametrize("mode,bucket_mb,world", [("allreduce", 0.05, 2), ("allreduce", 256.0, 2), ("zero1", 0.05, 2),
                                                   ("zero1", 256.0, 2), ("zero1", 0.05, 4), ("allreduce", 0.05, 4),
                                                   ("zero1", 0.05, 8)])
def test_ddp_grads_equal_single_process_global_batch(tmp_path, mode, bucket_mb, world):
    mp.start_processes(_worker, args=(world, _free_port(), str(tmp_path), bucket_mb, mode), nprocs=world,
                       start_method="spawn")
    gs = [torch.load(tmp_path / f"g{r}.pt") for r in range(world)]
    if mode == "allreduce":
        assert all(torch.equal(gs[0], g) for g in gs[1:])
        g0 = gs[0]
    else:  # the ranks own disjoint, complementary shards
        g0 = gs[0]
        for g in gs[1:]:
            assert not (~torch.isnan(g0) & ~torch.isnan(g)).any()
            g0 = torch.where(torch.isnan(g0), g, g0)
        assert not torch.isnan(g0).any()
    from fault_tolerant_llm_training_amd.data.synthetic import SyntheticTokens
    from fault_tolerant_llm_training_amd.models.llama import build_model, model_args_for

    a = model_args_for("tiny", vocab_size=128, seq_len=16)
    m = build_model(a, "cpu", torch.float32, seed=5)
    ds = SyntheticTokens(128, 16, seed=9, pin=False)
    x, y = ds.batch(1, 2 * world)  # global batch of the last step
    for r in range(world):
        y[2 * r, :3] = -100
    loss = m(x, y)
    loss.backward()
    assert torch.allclose(g0, m.flat.grads, atol=2e-6, rtol=1e-4)


def _torchrun(d, job, args, world=2):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "train.py")] + args
    env = env_for(d, job, {"OMP_NUM_THREADS": "1"})
    return cmd, env


def _run(d, job, args):
    cmd, env = _torchrun(d, job, args)
    r = subprocess.run(cmd, cwd=d, env=env, capture_output=True, text=True, timeout=600)
    return r.returncode, r.stdout + r.stderr


def _rank_pids(parent_pid):
    import psutil

    kids = psutil.Process(parent_pid).children(recursive=True)
    out = {}
    for k in kids:
        try:
            env = k.environ()
        except Exception:
            continue
        if "RANK" in env and "train.py" in " ".join(k.cmdline()):
            out[int(env["RANK"])] = k.pid
    return out


@pytest.mark.parametrize("mode", ["zero1", "allreduce"])
def test_dp_signal_to_one_rank_stops_all_and_resume_is_exact(tmp_path, mode):
    d = str(tmp_path)
    write_fake_sbatch(d)
    ck = ["--checkpoint-path", os.path.join(d, "ck")]
    base = TINY + ["--synthetic-data", "--vocab-size", "256", "--training-steps", "31", "--lr-warmup-steps", "3",
                   "--dp-mode", mode, "--dp-bucket-mb", "0.1"] + ck
    end = ["--raise-error", "--error-step", "30"]
    rc, out = _run(d, "100", base + end)
    assert rc == 0 and "Checkpoint saved at step 30" in out, out
    assert f"Data parallel over 2 ranks: {mode}" in out

    cmd, env = _torchrun(d, "200", base + end)
    log = open(os.path.join(d, "dp.log"), "w")
    p = subprocess.Popen(cmd, cwd=d, env=env, stdout=log, stderr=subprocess.STDOUT, start_new_session=True)
    try:
        assert wait_for_log(log.name, "Training step: 5 |", timeout=180), open(log.name).read()
        pids = {}
        for _ in range(100):
            pids = _rank_pids(p.pid)
            if len(pids) == 2:
                break
            time.sleep(0.1)
        assert set(pids) == {0, 1}
        os.kill(pids[1], signal.SIGUSR1)  # only rank 1 sees the signal
        assert p.wait(timeout=180) == 0
    finally:
        kill_group(p)
    out = open(log.name).read()
    # the logged loss is the global-batch mean (sum of the ranks' globally normalised losses),
    # not rank 0's half of it: ~ln(256) on random tokens
    lm = re.search(r"Training step: 5 \| Loss: ([0-9.]+)", out)
    assert lm and float(lm.group(1)) > 4.5, out
    m = re.search(r"Checkpoint saved at step (\d+)", out)
    assert m and "Job timed out" in out, out
    c = torch.load(os.path.join(d, "ck", "checkpoint_200.ckpt"), map_location="cpu", weights_only=True)
    assert c["training_step"] == int(m.group(1))
    assert isinstance(c["data_loader"], list) and len(c["data_loader"]) == 2
    assert all(s["next_step"] == c["training_step"] for s in c["data_loader"])
    assert c["meta"]["world_size"] == 2

    rc, out = _run(d, "300", base + end + ["--checkpoint-id", "200"])
    assert rc == 0 and f"Resuming training from training_step {c['training_step']}" in out, out
    a = torch.load(os.path.join(d, "ck", "checkpoint_100.ckpt"), map_location="cpu", weights_only=True)
    b = torch.load(os.path.join(d, "ck", "checkpoint_300.ckpt"), map_location="cpu", weights_only=True)
    for k in a["model"]:
        assert torch.equal(a["model"][k], b["model"][k]), k
    for i in a["optimizer"]["state"]:
        assert torch.equal(a["optimizer"]["state"][i]["exp_avg_sq"], b["optimizer"]["state"][i]["exp_avg_sq"])


def test_resume_dp2_checkpoint_on_one_rank_and_back(tmp_path):
    """The checkpoint is full-layout (ZeRO-1 shards are gathered), so the world size may change."""
    d = str(tmp_path)
    write_fake_sbatch(d)
    ck = ["--checkpoint-path", os.path.join(d, "ck")]
    base = TINY + ["--synthetic-data", "--vocab-size", "256", "--training-steps", "40", "--dp-bucket-mb", "0.1"] + ck
    rc, out = _run(d, "400", base + ["--raise-error", "--error-step", "6"])
    assert rc == 0 and "Checkpoint saved at step 6" in out, out
    from helpers import run_train

    rc, out = run_train(d, "401", base + ["--checkpoint-id", "400", "--raise-error", "--error-step", "9"])
    assert rc == 0 and "Resuming training from training_step 6" in out and "Checkpoint saved at step 9" in out, out
    assert "written by 2 ranks, resuming on 1" in out
    rc, out = _run(d, "402", base + ["--checkpoint-id", "401", "--raise-error", "--error-step", "12"])
    assert rc == 0 and "Resuming training from training_step 9" in out and "Checkpoint saved at step 12" in out, out


def _accum_worker(rank, world, port, out_dir, mode, K):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from fault_tolerant_llm_training_amd.data.synthetic import SyntheticTokens
    from fault_tolerant_llm_training_amd.models.llama import build_model, model_args_for
    from fault_tolerant_llm_training_amd.parallel.ddp import GradReducer

    a = model_args_for("tiny", vocab_size=128, seq_len=16)
    m = build_model(a, "cpu", torch.float32, seed=5)
    ddp = GradReducer(m.flat, m.sinks_in_backward_order(), bucket_mb=0.05, mode=mode)
    ds = SyntheticTokens(128, 16, seed=9, rank=rank, world_size=world, pin=False)
    x, y = ds.batch(0, K)  # this rank's K micro-batches of one sequence each
    y[0, :3] = -100
    n = torch.tensor([float((y != -100).sum())])
    dist.all_reduce(n)
    calls = []
    orig = ddp._launch_now
    ddp._launch_now = lambda b: (calls.append(b.idx), orig(b))[1]
    for k in range(K):
        ddp.begin_micro(k, K)
        loss = m(x[k : k + 1], y[k : k + 1], 1.0 / n)
        loss.backward()
        if k < K - 1:
            assert calls == [], "no collective before the last micro-batch"
    ddp.finish()
    assert calls == sorted(calls) and len(calls) == len(ddp.buckets), calls  # in-order launches
    full = torch.full_like(m.flat.grads, float("nan"))
    for b in ddp.buckets:
        if mode == "zero1" and not b.sparse:
            lo = b.lo + rank * b.shard_len
            full[lo : lo + b.shard_len] = ddp.grad_for_update(b)
        elif mode == "zero1":
            lo = b.lo + rank * b.shard_len
            full[lo : lo + b.shard_len] = m.flat.grads[lo : lo + b.shard_len]
        else:
            full[b.lo : b.hi] = m.flat.grads[b.lo : b.hi]
    torch.save(full, os.path.join(out_dir, f"a{rank}.pt"))
    dist.destroy_process_group()


@pytest.mark.parametrize("mode", ["allreduce", "zero1"])
def test_grad_accumulation_equals_global_batch(tmp_path, mode):
    """--grad-accum K: K micro-batches per rank, collectives only in the last backward (sparse
    embedding rows of all micro-batches exchanged at once) == one process on the global batch."""
    world, K = 2, 2
    mp.start_processes(_accum_worker, args=(world, _free_port(), str(tmp_path), mode, K), nprocs=world,
                       start_method="spawn")
    gs = [torch.load(tmp_path / f"a{r}.pt") for r in range(world)]
    g0 = gs[0]
    for g in gs[1:]:
        g0 = torch.where(torch.isnan(g0), g, g0)
    assert not torch.isnan(g0).any()
    from fault_tolerant_llm_training_amd.data.synthetic import SyntheticTokens
    from fault_tolerant_llm_training_amd.models.llama import build_model, model_args_for

    a = model_args_for("tiny", vocab_size=128, seq_len=16)
    m = build_model(a, "cpu", torch.float32, seed=5)
    xs, ys = [], []
    for r in range(world):
        x, y = SyntheticTokens(128, 16, seed=9, rank=r, world_size=world, pin=False).batch(0, K)
        y[0, :3] = -100
        xs.append(x)
        ys.append(y)
    loss = m(torch.cat(xs), torch.cat(ys))
    loss.backward()
    assert torch.allclose(g0, m.flat.grads, atol=2e-6, rtol=1e-4)
