"""Shared test utilities: subprocess runs of train.py, a fake ``sbatch``, tiny parquet files."""
from __future__ import annotations

import os
import signal
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TRAIN = os.path.join(ROOT, "train.py")

TINY = ["--device", "cpu", "--model", "tiny", "--sequence-length", "32", "--batch-size", "2",
        "--logging-frequency", "5", "--prefetch", "1"]


def write_fake_sbatch(d: str) -> str:
    """A ``sbatch`` stub: records its argv, prints Slurm's submit line."""
    path = os.path.join(d, "sbatch")
    with open(path, "w") as f:
        f.write("#!/bin/bash\n"
                f"echo \"$@\" >> {d}/sbatch_calls.txt\n"
                "echo \"Submitted batch job 424242\"\n")
    os.chmod(path, 0o755)
    return path


def sbatch_calls(d: str):
    p = os.path.join(d, "sbatch_calls.txt")
    if not os.path.exists(p):
        return []
    return [ln.split() for ln in open(p).read().splitlines() if ln.strip()]


def env_for(d: str, job_id: str, extra=None):
    env = dict(os.environ)
    env.update({"SLURM_JOB_ID": str(job_id), "WORKDIR": d, "PATH": d + os.pathsep + env.get("PATH", ""),
                "PYTHONUNBUFFERED": "1", "OMP_NUM_THREADS": "2"})
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "SLURM_PROCID", "SLURM_NTASKS"):
        env.pop(k, None)
    if extra:
        env.update(extra)
    return env


def run_train(d: str, job_id: str, args, timeout=300, extra_env=None):
    """Run train.py to completion; returns (returncode, combined output)."""
    r = subprocess.run([sys.executable, TRAIN] + list(args), cwd=d, env=env_for(d, job_id, extra_env),
                       capture_output=True, text=True, timeout=timeout)
    return r.returncode, r.stdout + r.stderr


def start_train(d: str, job_id: str, args, extra_env=None, log_name="run.log"):
    log = open(os.path.join(d, log_name), "w")
    p = subprocess.Popen([sys.executable, TRAIN] + list(args), cwd=d, env=env_for(d, job_id, extra_env),
                         stdout=log, stderr=subprocess.STDOUT, start_new_session=True)
    p._log_path = log.name  # type: ignore[attr-defined]
    return p


def wait_for_log(path: str, needle: str, timeout: float = 120.0) -> bool:
    t0 = time.time()
    while time.time() - t0 < timeout:
        if os.path.exists(path) and needle in open(path).read():
            return True
        time.sleep(0.05)
    return False


def kill_group(p):
    try:
        os.killpg(p.pid, signal.SIGKILL)
    except ProcessLookupError:
        pass


def make_parquet(path: str, n_docs: int = 40, seed: int = 0):
    import random

    import pyarrow as pa
    import pyarrow.parquet as pq

    rng = random.Random(seed)
    words = ["alpha", "beta", "gamma", "delta", "eps", "zeta", "eta", "theta", "iota", "kappa"]
    texts = [" ".join(rng.choice(words) for _ in range(rng.randint(2, 30))) for _ in range(n_docs)]
    pq.write_table(pa.table({"text": texts}), path)
    return texts
