#!/bin/bash
# Round 6, session Y: fp32 step A/B (gemm_f32 LDS-DMA form vs hipBLASLt), GPT-2-medium and Llama-3-8B.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 400 python -u scripts/ab_step.py --model gpt2-medium --vocab-size 50304 --dtype fp32 --knobs f32mfma \
  --rounds 4 --steps 10 > gpurun_out/r6y_ab_f32_gpt2-medium.log 2>&1 || { tail -5 gpurun_out/r6y_ab_f32_gpt2-medium.log; exit 1; }
grep "best" gpurun_out/r6y_ab_f32_gpt2-medium.log
timeout -k 10 600 python -u scripts/ab_step.py --model llama3-8b --dtype fp32 --knobs f32mfma \
  --rounds 3 --steps 4 --warmup 2 > gpurun_out/r6y_ab_f32_llama3-8b.log 2>&1 || { tail -5 gpurun_out/r6y_ab_f32_llama3-8b.log; exit 1; }
grep "best" gpurun_out/r6y_ab_f32_llama3-8b.log
