#!/bin/bash
# rocprofv3 kernel stats of the GPT-2 presets under the whole-step HIP graph (BASELINE configs 2-3)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for m in gpt2-small gpt2-medium; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$m -o run --output-format csv -- \
    python3 bench.py --model $m --graph --steps 20 --warmup 3 --no-ckpt > gpurun_out/prof_$m.log 2>&1 || exit $?
  tail -1 gpurun_out/prof_$m.log
done
for m in gpt2-small gpt2-medium; do
  timeout -k 10 300 python3 bench.py --model $m --graph --steps 50 --warmup 5 --no-ckpt > gpurun_out/bench_$m.log 2>&1 || exit $?
  tail -1 gpurun_out/bench_$m.log
done
