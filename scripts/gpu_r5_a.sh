#!/bin/bash
# Round 5, session A: 8B kernel trace (split-K dX in-tree), same-box split-K A/B, GPT-2 presets at
# vocab 50304 and 131072 under the whole-step HIP graph.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/prof8b
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof8b -o run --output-format csv -- python3 bench.py --steps 5 --warmup 3 --no-ckpt > gpurun_out/prof8b.log 2>&1 || exit 1
echo "prof ok"
timeout -k 10 400 python -u scripts/ab_step.py --knobs splitk --rounds 3 > gpurun_out/r5_ab_splitk.log 2>&1 || exit 1
echo "ab ok"
: > gpurun_out/r5_gpt2_bench.jsonl
for m in gpt2-small gpt2-medium; do
  for v in 50304 131072; do
    timeout -k 10 200 python -u bench.py --model $m --graph --vocab-size $v --steps 30 --warmup 5 --no-ckpt > gpurun_out/g_${m}_$v.log 2>&1 || { tail -5 gpurun_out/g_${m}_$v.log; exit 1; }
    tail -1 gpurun_out/g_${m}_$v.log >> gpurun_out/r5_gpt2_bench.jsonl
  done
done
echo "gpt2 ok"
