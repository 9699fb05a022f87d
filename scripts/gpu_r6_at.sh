#!/bin/bash
# Round 6, session AT: hardware queues per process (GPU_MAX_HW_QUEUES 4, the box default, vs 2) on the
# 8B bench step and the GPT-2-small graph step, alternating.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
for q in 4 2 4 2; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-ckpt > gpurun_out/r6at_b.json 2>gpurun_out/r6at_b.err || { tail -3 gpurun_out/r6at_b.err; exit 1; }
  echo "8b q=$q $(python3 -c "import json;d=json.loads(open('gpurun_out/r6at_b.json').read().strip().splitlines()[-1]);print(d['ms_per_step'], d.get('sclk_mhz_p50'))")" | tee -a gpurun_out/r6at.log
done
for q in 4 2 4 2; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python -u bench.py --model gpt2-small --vocab-size 50304 --graph --steps 50 --warmup 5 --no-ckpt > gpurun_out/r6at_b.json 2>gpurun_out/r6at_b.err || { tail -3 gpurun_out/r6at_b.err; exit 1; }
  echo "gpt2-small q=$q $(python3 -c "import json;d=json.loads(open('gpurun_out/r6at_b.json').read().strip().splitlines()[-1]);print(d['ms_per_step'], d.get('sclk_mhz_p50'))")" | tee -a gpurun_out/r6at.log
done
