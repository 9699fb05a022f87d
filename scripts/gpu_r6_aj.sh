#!/bin/bash
# Round 6, session AJ (final evidence): kernel stats of the 8B bench step and of the GPT-2-small graph
# step at HEAD.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
rm -rf gpurun_out/r6aj_p8 gpurun_out/r6aj_ps
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/r6aj_p8 -o run --output-format csv -- python3 bench.py --steps 8 --warmup 2 --no-ckpt > gpurun_out/r6aj_p8.log 2>&1 || exit 1
python scripts/prof_summary.py $(find gpurun_out/r6aj_p8 -name "run_kernel_stats.csv" | head -1) "Llama-3-8B bench step, round 6 final (10 steps incl. 2 warmup)" 10 > gpurun_out/r6aj_llama8b_kernel_stats.md
head -22 gpurun_out/r6aj_llama8b_kernel_stats.md
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r6aj_ps -o run --output-format csv -- python3 bench.py --model gpt2-small --vocab-size 50304 --graph --steps 20 --warmup 3 --no-ckpt > gpurun_out/r6aj_ps.log 2>&1 || exit 1
python scripts/prof_summary.py $(find gpurun_out/r6aj_ps -name "run_kernel_stats.csv" | head -1) "GPT-2-small vocab 50304 --graph, round 6 final (23 steps incl. warmup)" 23 > gpurun_out/r6aj_gpt2s_kernel_stats.md
head -22 gpurun_out/r6aj_gpt2s_kernel_stats.md
rm -rf gpurun_out/r6aj_p8 gpurun_out/r6aj_ps
