#!/bin/bash
# Round 6, session AH: fp32 steps (gemm_f32): the dW side stream on / off.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
for m in gpt2-small gpt2-medium; do
  timeout -k 10 400 python -u scripts/ab_step.py --model $m --vocab-size 50304 --dtype fp32 --knobs dw \
    --rounds 4 --steps 10 > gpurun_out/r6ah_ab_dw_$m.log 2>&1 || { tail -5 gpurun_out/r6ah_ab_dw_$m.log; exit 1; }
  grep "best" gpurun_out/r6ah_ab_dw_$m.log
done
