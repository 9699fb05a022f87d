#!/usr/bin/env python3
"""Preempt → save → resubmit → resume chain benchmark (BASELINE configs 2/4/5).

Runs ``train.sh`` under the local Slurm emulator (``ft.slurm_sim``): each job gets
SIGUSR1 ``--signal-lead`` seconds before ``--time``; train.py saves, resubmits itself
with its job id, and the next job resumes. Prints one JSON line with, per job: the
step it resumed from, the step it saved, the save wall-clock, the setup time of a
resumed job, and the chain's steps lost (must be 0) — the quantities the reference
only shows in its Slurm logs (save 33.6 s, resume setup 60.6 s).

    python benchmarks/preempt_chain.py --jobs 3 --time 90 --signal-lead 30 -- \
        --model gpt2-small --synthetic-data --sequence-length 2048
"""
from __future__ import annotations

import argparse
import json
import os
import re
import sys
import tempfile
from datetime import datetime

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from fault_tolerant_llm_training_amd.ckpt.format import checkpoint_file  # noqa: E402
from fault_tolerant_llm_training_amd.ft.slurm_sim import SlurmSim  # noqa: E402

TS = re.compile(r"^(\d{4}-\d\d-\d\d \d\d:\d\d:\d\d,\d{3}) - ")


def _t(line):
    m = TS.match(line)
    return datetime.strptime(m.group(1), "%Y-%m-%d %H:%M:%S,%f").timestamp() if m else None


def parse(log):
    lines = open(log).read().splitlines()
    out = {"resumed_from": None, "saved_at": None, "save_s": None, "setup_s": None, "requeued": False,
           "last_step": None}
    t_args = t_start = t_handler = t_saved = None
    for ln in lines:
        t = _t(ln)
        if "Experiment args:" in ln:
            t_args = t
        m = re.search(r"Resuming training from training_step (\d+)", ln)
        if m:
            out["resumed_from"] = int(m.group(1))
            t_start = t
        if "Starting training!" in ln:
            t_start = t
        m = re.search(r"Training step: (\d+) \|", ln)
        if m:
            out["last_step"] = int(m.group(1))
        if "[EXIT HANDLER] Job timed out" in ln:
            t_handler = t
        m = re.search(r"Checkpoint saved at step (\d+)", ln)
        if m:
            out["saved_at"] = int(m.group(1))
            t_saved = t
        if "sbatch requeued" in ln:
            out["requeued"] = True
    if t_args and t_start:
        out["setup_s"] = round(t_start - t_args, 2)
    if t_handler and t_saved:
        out["save_s"] = round(t_saved - t_handler, 2)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--jobs", type=int, default=3)
    ap.add_argument("--time", type=float, default=90.0)
    ap.add_argument("--signal-lead", type=float, default=30.0)
    ap.add_argument("--workdir", default=ROOT)
    ap.add_argument("--checkpoint-path", default="")
    ap.add_argument("--log-dir", default="", help="where the jobs' output_<JOBID>.out go (default: a temp dir)")
    ap.add_argument("--prune-consumed", action="store_true",
                    help="delete a job's checkpoint once the next job has resumed from it AND written a "
                         "durable checkpoint of its own (an 8B chain holds at most two 48 GB checkpoints "
                         "on disk instead of one per job, and always one it can resume from)")
    ap.add_argument("--prune-on-resume", action="store_true",
                    help="delete a job's checkpoint as soon as the next job has resumed from it (a disk "
                         "that holds ONE checkpoint, e.g. 79 GB for the 48 GB 8B file: the next save "
                         "needs the space; a job that dies before its own save then has nothing to "
                         "resume from -- the trade --prune-consumed avoids where two fit)")
    ap.add_argument("--rotate", default="",
                    help="a second checkpoint directory (another filesystem): train.py --checkpoint-alt-path DIR "
                         "--prune-consumed -- each job writes to the directory it did not resume from and "
                         "deletes its predecessor's file only once its own is durable, so a disk with room for "
                         "ONE checkpoint still always holds a complete one (the other tier holds the other)")
    ap.add_argument("train_args", nargs=argparse.REMAINDER)
    a = ap.parse_args()
    extra = [x for x in a.train_args if x != "--"]
    ck = a.checkpoint_path or tempfile.mkdtemp(prefix="ftck_")
    dirs = [ck] + ([a.rotate] if a.rotate else [])
    for d_ in dirs:
        os.makedirs(d_, exist_ok=True)
    env = dict(os.environ)
    rot = ["--checkpoint-alt-path", a.rotate, "--prune-consumed"] if a.rotate else []
    env["EXTRA_TRAINING_ARGS"] = " ".join(extra + ["--training-steps", "100000000", "--error-step", "100000000",
                                                   "--checkpoint-path", ck] + rot)
    env.setdefault("PYTHONUNBUFFERED", "1")
    logdir = a.log_dir or tempfile.mkdtemp(prefix="ftlogs_")
    os.makedirs(logdir, exist_ok=True)
    sim = SlurmSim(a.workdir, a.time, a.signal_lead, kill_wait=30.0, env=env, log_dir=logdir)
    sim.submit("train.sh")
    pruned = []

    def prune(rec):
        # the running job resumed from its predecessor's checkpoint and has since made its own
        # durable (a periodic save's "Checkpoint written" or the exit handler's "Checkpoint saved",
        # both logged after the atomic rename): only then is the predecessor's file not needed --
        # a job that dies before its first save is resumed from the predecessor's again
        if not sim.jobs or sim.jobs[-1].job_id in pruned:
            return
        prev = sim.jobs[-1].job_id
        try:
            with open(rec.log) as f:
                text = f.read()
        except OSError:
            return
        resumed = "Resuming training from training_step" in text
        own = "Checkpoint written:" in text or "[EXIT HANDLER] Checkpoint saved at step" in text
        if resumed and (own or a.prune_on_resume):
            path = checkpoint_file(ck, prev)
            if os.path.exists(path):
                os.remove(path)
            pruned.append(prev)

    # complete checkpoint files (atomically renamed *.ckpt) over every directory, sampled every poll
    # (50 ms) while a job runs: after the first one exists the chain must never hold zero
    durable = {"min": None, "max": 0, "samples": 0}

    def count_durable():
        n = 0
        for d_ in dirs:
            try:
                n += sum(1 for f in os.listdir(d_) if f.startswith("checkpoint_") and f.endswith(".ckpt"))
            except OSError:
                pass
        durable["max"] = max(durable["max"], n)
        if n or durable["min"] is not None:
            durable["min"] = n if durable["min"] is None else min(durable["min"], n)
            durable["samples"] += 1

    def hook(rec):
        if a.prune_consumed or a.prune_on_resume:
            prune(rec)
        count_durable()

    jobs = sim.run(a.jobs, hook)
    count_durable()
    rows, lost = [], 0
    prev = None
    for j in jobs:
        r = parse(j.log)
        r.update(job=j.job_id, rc=j.returncode, signals=j.signals, wall_s=round(j.seconds, 1))
        if prev is not None and prev.get("saved_at") is not None and r["resumed_from"] is not None:
            lost += r["resumed_from"] - prev["saved_at"]
        rows.append(r)
        prev = r
    print(json.dumps({"benchmark": "preempt_chain", "args": extra, "time_limit_s": a.time,
                      "signal_lead_s": a.signal_lead, "jobs": rows, "steps_lost": lost,
                      "pruned_checkpoints": pruned,
                      "checkpoint_dirs": dirs,
                      "final_checkpoints": {d_: sorted(os.listdir(d_)) for d_ in dirs},
                      "durable_checkpoints_min_after_first": durable["min"],
                      "durable_checkpoints_max": durable["max"], "durable_samples": durable["samples"],
                      "logs": logdir}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
