"""bench.py driver contract (single JSON line, whole-job value, max over ranks) on CPU/gloo.

The driver runs ``python bench.py`` for N=1 and ``torch.distributed.run ... bench.py --gpus N``
for N>1; this exercises the same code path (process groups, gradient reducer modes, barriers,
max-over-ranks timing) with gloo and a tiny model.
"""
import json
import os
import socket
import subprocess
import sys

import pytest

from helpers import ROOT

pytestmark = pytest.mark.slow

ARGS = ["--device", "cpu", "--model", "tiny", "--vocab-size", "256", "--seq-len", "64", "--steps", "2",
        "--warmup", "1", "--bucket-mb", "0.1"]


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _env(ckpt_dir=None):
    env = dict(os.environ)
    env["OMP_NUM_THREADS"] = "1"
    if ckpt_dir is not None:
        env["FT_BENCH_CKPT_DIR"] = str(ckpt_dir)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
        env.pop(k, None)
    return env


def _json_lines(out):
    return [json.loads(ln) for ln in out.splitlines() if ln.startswith("{")]


def _check_ckpt(j, world):
    """The checkpoint-save block (second half of the BASELINE metric) ran without error; under DP
    every rank ran the same loaded steps (a mismatch would have hung the collectives)."""
    c = j["ckpt_save"]
    assert "error" not in c, c
    assert c["exit_save_s"] > 0 and c["bytes"] > 0
    assert c["loaded"]["steps_until_durable"] >= 3 and c["loaded"]["save_to_durable_s"] is not None


def test_bench_single_process_json(tmp_path):
    r = subprocess.run([sys.executable, "bench.py"] + ARGS, cwd=ROOT, env=_env(tmp_path), capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    lines = _json_lines(r.stdout)
    assert len(lines) == 1
    j = lines[0]
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config"):
        assert k in j, k
    assert j["n_gpus"] == 1 and j["steps"] == 2 and j["config"]["parallelism"] == "dp1"
    assert abs(j["value"] - 64 / (j["ms_per_step"] / 1e3)) / j["value"] < 0.02
    _check_ckpt(j, 1)


@pytest.mark.parametrize("mode", ["zero1", "allreduce"])
def test_bench_torchrun_two_ranks(mode, tmp_path):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(_port()), "bench.py", "--gpus", "2", "--dp-mode", mode] + ARGS
    r = subprocess.run(cmd, cwd=ROOT, env=_env(tmp_path), capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1, r.stdout  # rank 0 only
    j = lines[0]
    assert j["n_gpus"] == 2 and j["config"]["parallelism"] == "dp2" and j["config"]["global_batch"] == 2
    assert j["grad_mode"] == mode
    assert abs(j["value"] - 2 * 64 / (j["ms_per_step"] / 1e3)) / j["value"] < 0.02
    # vs_baseline is per GPU (the metric is tokens/sec/GPU): it does not scale with N by itself
    assert abs(j["vs_baseline"] - j["tokens_per_s_per_gpu"] / 6376.0) < 1e-3
    assert "exposed_comm_ms_per_step" in j and "compute_only_ms_per_step" in j
    _check_ckpt(j, 2)


def test_bench_grad_accum_two_ranks():  # (no checkpoint block: --no-ckpt)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(_port()), "bench.py", "--gpus", "2", "--grad-accum", "2", "--no-ckpt"] + ARGS
    r = subprocess.run(cmd, cwd=ROOT, env=_env(), capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    j = _json_lines(r.stdout)[0]
    assert j["config"]["global_batch"] == 4 and j["grad_accum"] == 2
    assert abs(j["value"] - 4 * 64 / (j["ms_per_step"] / 1e3)) / j["value"] < 0.02


@pytest.mark.parametrize("world", [4, 8])
def test_bench_torchrun_n_ranks_zero1(world, tmp_path):
    """Rehearsal of the driver's N = 4 / 8 runs (one process per GPU there; gloo ranks here): the
    default ZeRO-1 mode with 64-element-aligned shards, the sparse embedding exchange across all
    ranks, the exposed-communication re-timing and the sharded checkpoint block."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(world),
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), "bench.py", "--gpus", str(world)] + ARGS
    r = subprocess.run(cmd, cwd=ROOT, env=_env(tmp_path), capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1, r.stdout
    j = lines[0]
    assert j["n_gpus"] == world and j["config"]["parallelism"] == f"dp{world}"
    assert j["config"]["global_batch"] == world and j["grad_mode"] == "zero1"
    assert abs(j["value"] - world * 64 / (j["ms_per_step"] / 1e3)) / j["value"] < 0.02
    assert "exposed_comm_ms_per_step" in j and j["comm_GB_per_rank_per_step"] >= 0
    # self-validation fields of the driver's multi-GPU run: the process group's real size and
    # every rank's device (on GPUs: one distinct device per rank, else bench.py raises)
    assert j["world_size"] == world and len(j["device_ids"]) == world
    assert j["distinct_devices"] >= 1 and "peer_access_all_pairs" in j and "rccl_version" in j
    _check_ckpt(j, world)


def test_bench_self_launch_without_launcher(tmp_path):
    """``python bench.py --gpus 4`` with no torchrun / Slurm variables starts 4 ranks itself (a child
    torchrun, never an exec) and reports a 4-rank measurement."""
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "4", "--no-ckpt", "--no-exposed-comm"] + ARGS, cwd=ROOT,
                       env=_env(tmp_path), capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1, r.stdout
    j = lines[0]
    assert j["n_gpus"] == 4 and j["world_size"] == 4 and j["config"]["parallelism"] == "dp4"
    assert len(j["device_ids"]) == 4


def test_bench_world_mismatch_fails():
    """A launcher that started a different number of ranks than ``--gpus`` is an error (rc != 0),
    never a silently relabelled number."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(_port()), "bench.py", "--gpus", "3", "--no-ckpt"] + ARGS
    r = subprocess.run(cmd, cwd=ROOT, env=_env(), capture_output=True, text=True, timeout=300)
    assert r.returncode != 0
    assert not _json_lines(r.stdout)
    assert "launcher started 2" in r.stderr
