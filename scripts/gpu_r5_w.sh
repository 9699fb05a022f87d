#!/bin/bash
# Round 5, session W: long-context throughput at HEAD + GPT-2-small kernel stats (graph step).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
bash scripts/gpu_long_context.sh > gpurun_out/r5w_long.log 2>&1 || { tail -5 gpurun_out/r5w_long.log; exit 1; }
rm -rf gpurun_out/prof_w && mkdir -p gpurun_out/prof_w
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_w -o run --output-format csv -- python3 bench.py --model gpt2-small --vocab-size 50304 --graph --steps 20 --warmup 3 --no-ckpt > gpurun_out/r5w_prof.log 2>&1 || exit 1
python3 -c "
import json
for l in open('gpurun_out/r5w_long.log'):
    l=l.strip()
    if l.startswith('{'):
        d=json.loads(l); print(d['config']['seq_len'], d['ms_per_step'], d['value'])
"
