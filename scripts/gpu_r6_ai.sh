#!/bin/bash
# Round 6, session AI: fp32 split-K reduction over 4 workgroups per tile (no partials): tests, fp32 step A/B.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_gemm_f32_gpu.py > gpurun_out/r6ai_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r6ai_tests.log; [ $rc -eq 0 ] || exit $rc
for m in gpt2-small gpt2-medium; do
  timeout -k 10 400 python -u scripts/ab_step.py --model $m --vocab-size 50304 --dtype fp32 --knobs f32mfma \
    --rounds 4 --steps 10 > gpurun_out/r6ai_ab_f32_$m.log 2>&1 || { tail -5 gpurun_out/r6ai_ab_f32_$m.log; exit 1; }
  grep "best" gpurun_out/r6ai_ab_f32_$m.log
done
