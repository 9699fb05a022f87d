"""The data-parallel path over RCCL on the GPU (1-rank process group, explicit DP mode).

A single-GPU box cannot host two RCCL ranks (one GPU per rank), so this runs bench.py under
torchrun with one rank and an explicit ``--dp-mode``: the gradient buckets then really go
through RCCL reduce-scatter / all-reduce / all-gather issued from the dW side stream and
the optimizer stream, the sparse embedding exchange all-gathers through RCCL, and the
step must produce the same loss as the local (no collective) run of the same seed.
The multi-rank logic is covered by the gloo tests (test_dp_gloo.py, test_bench_contract.py).
"""
import json
import os
import socket
import subprocess
import sys

import pytest

from helpers import ROOT

pytestmark = pytest.mark.gpu

ARGS = ["--model", "tiny", "--vocab-size", "4096", "--seq-len", "256", "--steps", "3", "--warmup", "1",
        "--bucket-mb", "0.5"]


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(extra, torchrun):
    env = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
        env.pop(k, None)
    env["HSA_ENABLE_IPC_MODE_LEGACY"] = "0"
    if torchrun:
        env["FT_FORCE_DIST"] = "1"  # build the RCCL process group even for one rank
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
               "--master-addr", "127.0.0.1", "--master-port", str(_port()), "bench.py", "--gpus", "1"]
    else:
        cmd = [sys.executable, "bench.py"]
    r = subprocess.run(cmd + ARGS + extra, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [json.loads(ln) for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    return lines[0]


@pytest.mark.parametrize("mode,rdt", [("zero1", "native"), ("allreduce", "native"), ("zero1", "fp32"),
                                      ("allreduce", "fp32")])
def test_rccl_one_rank_matches_local(mode, rdt):
    """fp32: the reduced fp32 copy is written back from the reducer's side stream while its
    buffers were allocated on the launching stream (record_stream keeps them alive)."""
    local = _run([], torchrun=False)
    dp = _run(["--dp-mode", mode, "--dp-reduce-dtype", rdt], torchrun=True)
    assert dp["grad_mode"] == mode and local["grad_mode"] == "local"
    assert dp["world_size"] == 1 and dp["distinct_devices"] == 1
    # same math: the 1-rank collectives are identities; zero1 shards are the whole buckets
    assert abs(dp["final_loss"] - local["final_loss"]) < 1e-3, (dp["final_loss"], local["final_loss"])


@pytest.mark.parametrize("mode", ["zero1", "allreduce"])
def test_rccl_one_rank_graph_matches_eager(mode):
    """The whole-step HIP graph under data parallelism: the bucket reduce-scatters / all-reduces and
    (ZeRO-1) the norm all-reduce and the parameter all-gathers are captured into the graph; replays
    give the same loss as the eager DP steps (reference --compile, train.py:61-63). ZeRO-1 under
    capture crashed while its collectives ran on two streams (RCCL collectives captured on more than
    one stream segfault hipStreamEndCapture: scripts/capture_collectives_probe.py); under the graph
    they are all issued blocking on the reducer's side stream (GradReducer.single_stream)."""
    eager = _run(["--dp-mode", mode, "--no-ckpt"], torchrun=True)
    graph = _run(["--dp-mode", mode, "--no-ckpt", "--graph"], torchrun=True)
    assert graph.get("hip_graph") is True and graph["grad_mode"] == mode and graph["world_size"] == 1
    assert abs(graph["final_loss"] - eager["final_loss"]) < 1e-6, (graph["final_loss"], eager["final_loss"])


def test_train_py_compile_under_dp(tmp_path):
    """train.py --compile on a (1-rank, RCCL) process group in the all-reduce mode and in the default
    ZeRO-1 mode: the step runs as the whole-step HIP graph with the collectives inside, and training
    completes."""
    from helpers import run_train, write_fake_sbatch

    d = str(tmp_path)
    write_fake_sbatch(d)
    env = {"RANK": "0", "WORLD_SIZE": "1", "LOCAL_RANK": "0", "MASTER_ADDR": "127.0.0.1",
           "MASTER_PORT": str(_port()), "FT_FORCE_DIST": "1", "HSA_ENABLE_IPC_MODE_LEGACY": "0"}
    args = ["--device", "cuda", "--model", "tiny", "--synthetic-data", "--vocab-size", "1024", "--sequence-length",
            "256", "--batch-size", "2", "--compile", "--dp-mode", "allreduce", "--logging-frequency", "5",
            "--checkpoint-path", os.path.join(d, "ck"), "--training-steps", "12"]
    rc, out = run_train(d, "795", args, timeout=240, extra_env=env)
    assert rc == 0 and "Using `torch.compile`" in out and "HIP graph" in out, out[-3000:]
    assert "Training completed" in out, out[-3000:]
    env["MASTER_PORT"] = str(_port())
    rc, out = run_train(d, "796", [x if x != "allreduce" else "zero1" for x in args], timeout=240, extra_env=env)
    assert rc == 0 and "not applied" not in out and "HIP graph:" in out and "Training completed" in out, out[-3000:]
    assert "Data parallel over 1 ranks: zero1" in out, out[-3000:]


def _ckpt(d, job):
    import torch

    return torch.load(os.path.join(d, "ck", f"checkpoint_{job}.ckpt"), map_location="cpu", weights_only=True)


def _same_state(a, b):
    import torch

    assert a["training_step"] == b["training_step"]
    for k in a["model"]:
        assert torch.equal(a["model"][k], b["model"][k]), k
    for i in a["optimizer"]["state"]:
        sa, sb = a["optimizer"]["state"][i], b["optimizer"]["state"][i]
        assert float(sa["step"]) == float(sb["step"]), i
        assert torch.equal(sa["exp_avg"], sb["exp_avg"]) and torch.equal(sa["exp_avg_sq"], sb["exp_avg_sq"]), i


def test_graph_dp_faults_save_the_state_before_the_failed_step(tmp_path):
    """--compile under data parallelism (whole-step HIP graph, all-reduce mode, 1-rank RCCL group):

    * an OSError in this rank's forward (FT_INJECT_FAULT=0:6:forward) fires before the replay; the
      replay runs poisoned (NaN loss scale, so every captured collective carries NaN and the peers'
      replays complete), the non-finite guard skips the update, the vote stops at step 6 and the
      checkpoint equals the one an injected error at the step-6 boundary writes;
    * a lost peer at the step-6 boundary (FT_INJECT_FAULT=0:6:peerloss: the vote raises) leaves the
      last replay's optimizer step pending; the survivor completes it before its solo save, so the
      file records step 6 with all six updates (not five), bit-identical to the two above."""
    from helpers import run_train, write_fake_sbatch

    d = str(tmp_path)
    write_fake_sbatch(d)
    args = ["--device", "cuda", "--model", "tiny", "--synthetic-data", "--vocab-size", "1024", "--sequence-length",
            "256", "--batch-size", "2", "--learning-rate", "1e-3", "--lr-warmup-steps", "3", "--compile",
            "--dp-mode", "allreduce", "--logging-frequency", "5", "--checkpoint-path", os.path.join(d, "ck"),
            "--training-steps", "12"]

    def env(fault=""):
        e = {"RANK": "0", "WORLD_SIZE": "1", "LOCAL_RANK": "0", "MASTER_ADDR": "127.0.0.1",
             "MASTER_PORT": str(_port()), "FT_FORCE_DIST": "1", "HSA_ENABLE_IPC_MODE_LEGACY": "0"}
        if fault:
            e["FT_INJECT_FAULT"] = fault
        return e

    rc, out = run_train(d, "810", args + ["--raise-error", "--error-step", "6"], timeout=240, extra_env=env())
    assert rc == 0 and "HIP graph:" in out and "Checkpoint saved at step 6" in out, out[-3000:]
    rc, out = run_train(d, "811", args, timeout=240, extra_env=env("0:6:forward"))
    assert rc == 0 and "(forward, graph mode)" in out and "Checkpoint saved at step 6" in out, out[-3000:]
    rc, out = run_train(d, "812", args, timeout=240, extra_env=env("0:6:peerloss"))
    assert rc == 1 and "Lost a peer rank" in out and "Checkpoint saved at step 6" in out, out[-3000:]
    ref = _ckpt(d, 810)
    _same_state(ref, _ckpt(d, 811))
    _same_state(ref, _ckpt(d, 812))
