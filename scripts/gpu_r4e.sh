#!/bin/bash
# GPT-2-small step profile (small-model efficiency)
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/kprof_g2s
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/kprof_g2s -o run --output-format csv -- python3 bench.py --model gpt2-small --steps 10 --warmup 3 > gpurun_out/kprof_g2s.log 2>&1 || exit 1
tail -1 gpurun_out/kprof_g2s.log
