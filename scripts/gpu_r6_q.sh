#!/bin/bash
# Round 6, session Q: fp32 MFMA GEMM with the fragment reads pipelined across the barrier:
# numerics, products vs hipBLASLt, fp32 step A/B.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_gemm_f32_gpu.py > gpurun_out/r6q_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r6q_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/gemm_f32_bench.py > gpurun_out/r6q_f32_bench.log 2>&1 || { tail -5 gpurun_out/r6q_f32_bench.log; exit 1; }
cat gpurun_out/r6q_f32_bench.log
timeout -k 10 400 python -u scripts/ab_step.py --model gpt2-small --vocab-size 50304 --dtype fp32 --knobs f32mfma \
  --rounds 4 --steps 10 > gpurun_out/r6q_ab_f32_gpt2-small.log 2>&1 || { tail -5 gpurun_out/r6q_ab_f32_gpt2-small.log; exit 1; }
grep "best" gpurun_out/r6q_ab_f32_gpt2-small.log
