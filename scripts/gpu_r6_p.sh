#!/bin/bash
# Round 6, session P: fp32 model steps with the GEMMs on the fp32 MFMA kernel vs hipBLASLt (same
# process, alternating windows), GPT-2-small / -medium (V = 50304) and Llama-3-8B.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
for m in gpt2-small gpt2-medium; do
  timeout -k 10 400 python -u scripts/ab_step.py --model $m --vocab-size 50304 --dtype fp32 --knobs f32mfma \
    --rounds 4 --steps 10 > gpurun_out/r6p_ab_f32_$m.log 2>&1 || { tail -5 gpurun_out/r6p_ab_f32_$m.log; exit 1; }
  grep "best\|final" gpurun_out/r6p_ab_f32_$m.log
done
timeout -k 10 600 python -u scripts/ab_step.py --model llama3-8b --dtype fp32 --knobs f32mfma \
  --rounds 3 --steps 4 --warmup 2 > gpurun_out/r6p_ab_f32_llama3-8b.log 2>&1 || { tail -5 gpurun_out/r6p_ab_f32_llama3-8b.log; exit 1; }
grep "best\|final" gpurun_out/r6p_ab_f32_llama3-8b.log
