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


@pytest.mark.parametrize("mode", ["allreduce"])
def test_rccl_one_rank_graph_matches_eager(mode):
    """The whole-step HIP graph under data parallelism: the bucket all-reduces and the sparse
    embedding all-gather are captured into the graph; replays give the same loss as the eager DP
    steps (reference --compile, train.py:61-63). (ZeRO-1's gated parameter all-gathers crashed
    under capture: --graph refuses that mode.)"""
    eager = _run(["--dp-mode", mode, "--no-ckpt"], torchrun=True)
    graph = _run(["--dp-mode", mode, "--no-ckpt", "--graph"], torchrun=True)
    assert graph.get("hip_graph") is True and graph["grad_mode"] == mode and graph["world_size"] == 1
    assert abs(graph["final_loss"] - eager["final_loss"]) < 1e-6, (graph["final_loss"], eager["final_loss"])


def test_train_py_compile_under_dp(tmp_path):
    """train.py --compile on a (1-rank, RCCL) process group in the all-reduce mode: the step runs as
    the whole-step HIP graph with the collectives inside, and training completes; under ZeRO-1
    --compile is accepted and logged as not applied."""
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
    assert rc == 0 and "not applied" in out and "HIP graph:" not in out and "Training completed" in out, out[-3000:]
