"""A local Slurm emulator for the resubmit chain (tests and single-box demos).

The reference's fault tolerance is a *job chain* driven by Slurm (SURVEY.md
§3.3-3.5, §5.3): ``#SBATCH --signal=USR1@120`` delivers SIGUSR1 120 s before
``--time``; ``train.py`` saves and runs ``sbatch $WORKDIR/train.sh $JOBID``;
the next job gets the old id as ``$1`` and resumes; ``scancel`` sends
SIGTERM; at the time limit Slurm sends SIGTERM, then SIGKILL after
``KillWait``. No Slurm exists on the dev box or the GPU box, so this module
emulates exactly that contract:

* ``sbatch`` / ``srun`` shims are put first on ``PATH``: ``sbatch`` enqueues
  (script, args) and prints ``Submitted batch job <id>``; ``srun`` runs its
  command (``exec srun --unbuffered python train.py …`` works unchanged);
* each job runs ``bash <script> [args]`` in its own process group with
  ``SLURM_JOB_ID`` set and stdout to ``output_<id>.out``;
* at ``time_limit - signal_lead`` the job's processes get SIGUSR1, at
  ``time_limit`` SIGTERM, ``kill_wait`` later SIGKILL (``--no-requeue``:
  nothing is requeued unless the job itself calls ``sbatch``);
* jobs run one after another until the queue is empty or ``max_jobs``.

    python -m fault_tolerant_llm_training_amd.ft.slurm_sim --time 60 --signal-lead 20 \
        --max-jobs 3 --workdir /path/to/repo -- train.sh
"""
from __future__ import annotations

import argparse
import json
import os
import signal
import subprocess
import sys
import tempfile
import time
from dataclasses import dataclass, field
from typing import List, Optional

_SBATCH = """#!/bin/bash
# emulated sbatch: enqueue and print the Slurm submit line
Q="{queue}"
exec 9>>"$Q.lock"
flock 9
N=$(( $(cat "{counter}") + 1 ))
echo $N > "{counter}"
python3 -c 'import json,sys; print(json.dumps({{"id": int(sys.argv[1]), "argv": sys.argv[2:]}}))' "$N" "$@" >> "$Q"
echo "Submitted batch job $N"
"""

_SRUN = """#!/bin/bash
# emulated srun: drop srun options, run the task in place
while [[ "$1" == --* ]]; do shift; done
exec "$@"
"""


@dataclass
class JobRecord:
    job_id: int
    argv: List[str]
    returncode: Optional[int] = None
    signals: List[str] = field(default_factory=list)
    seconds: float = 0.0
    log: str = ""


class SlurmSim:
    def __init__(self, workdir: str, time_limit: float, signal_lead: float, kill_wait: float = 30.0,
                 first_job_id: int = 1000, env: Optional[dict] = None, log_dir: Optional[str] = None):
        self.workdir = os.path.abspath(workdir)
        self.time_limit = time_limit
        self.signal_lead = signal_lead
        self.kill_wait = kill_wait
        self.state = tempfile.mkdtemp(prefix="slurm_sim_")
        self.log_dir = log_dir or self.workdir
        self.queue = os.path.join(self.state, "queue.jsonl")
        self.counter = os.path.join(self.state, "counter")
        with open(self.counter, "w") as f:
            f.write(str(first_job_id - 1))
        open(self.queue, "w").close()
        self.bin = os.path.join(self.state, "bin")
        os.makedirs(self.bin)
        for name, body in (("sbatch", _SBATCH.format(queue=self.queue, counter=self.counter)), ("srun", _SRUN)):
            p = os.path.join(self.bin, name)
            with open(p, "w") as f:
                f.write(body)
            os.chmod(p, 0o755)
        self.env = dict(os.environ if env is None else env)
        self.env["PATH"] = self.bin + os.pathsep + self.env.get("PATH", "")
        self.env["WORKDIR"] = self.workdir
        self.env.pop("FT_SBATCH", None)
        self._consumed = 0
        self.jobs: List[JobRecord] = []

    def submit(self, script: str, *args: str) -> int:
        r = subprocess.run(["sbatch", script, *args], env=self.env, capture_output=True, text=True, check=True)
        return int(r.stdout.strip().split()[-1])

    def _pop(self) -> Optional[dict]:
        lines = [ln for ln in open(self.queue).read().splitlines() if ln.strip()]
        if self._consumed >= len(lines):
            return None
        req = json.loads(lines[self._consumed])
        self._consumed += 1
        return req

    def _signal(self, p: subprocess.Popen, sig: int, rec: JobRecord):
        rec.signals.append(signal.Signals(sig).name)
        try:
            os.killpg(p.pid, sig)
        except ProcessLookupError:
            pass

    def run_job(self, req: dict, hook=None) -> JobRecord:
        """Runs one queued job to its end; ``hook(rec)`` is called every poll (50 ms) while it runs."""
        jid, argv = req["id"], req["argv"]
        rec = JobRecord(jid, argv, log=os.path.join(self.log_dir, f"output_{jid}.out"))
        env = dict(self.env)
        env["SLURM_JOB_ID"] = str(jid)
        env["SLURM_SUBMIT_DIR"] = self.workdir
        script = argv[0] if os.path.isabs(argv[0]) else os.path.join(self.workdir, argv[0])
        t0 = time.monotonic()
        with open(rec.log, "w") as log:
            p = subprocess.Popen(["bash", script, *argv[1:]], cwd=self.workdir, env=env, stdout=log,
                                 stderr=subprocess.STDOUT, start_new_session=True)
            usr1_at = self.time_limit - self.signal_lead
            stage = 0
            while p.poll() is None:
                el = time.monotonic() - t0
                if stage == 0 and el >= usr1_at:
                    self._signal(p, signal.SIGUSR1, rec)
                    stage = 1
                elif stage == 1 and el >= self.time_limit:
                    self._signal(p, signal.SIGTERM, rec)
                    stage = 2
                elif stage == 2 and el >= self.time_limit + self.kill_wait:
                    self._signal(p, signal.SIGKILL, rec)
                    stage = 3
                if hook is not None:
                    hook(rec)
                time.sleep(0.05)
        rec.returncode = p.returncode
        rec.seconds = time.monotonic() - t0
        self.jobs.append(rec)
        return rec

    def run(self, max_jobs: int = 10, hook=None) -> List[JobRecord]:
        while len(self.jobs) < max_jobs:
            req = self._pop()
            if req is None:
                break
            self.run_job(req, hook)
        return self.jobs


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--time", type=float, required=True, help="job time limit in seconds (#SBATCH --time)")
    ap.add_argument("--signal-lead", type=float, default=120.0, help="USR1 lead in seconds (--signal=USR1@N)")
    ap.add_argument("--kill-wait", type=float, default=30.0)
    ap.add_argument("--max-jobs", type=int, default=3)
    ap.add_argument("--workdir", default=os.getcwd())
    ap.add_argument("script", nargs=argparse.REMAINDER)
    a = ap.parse_args(argv)
    script = [s for s in a.script if s != "--"]
    sim = SlurmSim(a.workdir, a.time, a.signal_lead, a.kill_wait)
    sim.submit(*script)
    for r in sim.run(a.max_jobs):
        print(json.dumps(r.__dict__), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
