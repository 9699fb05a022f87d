#!/bin/bash
# Round 6, session N: the fp32 MFMA GEMM (gemm_f32.hip): numerics, fp32 model step parity, kernel vs
# hipBLASLt on the fp32 products, and an fp32 GPT-2-small bench with its kernel trace.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r6n_prof
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_gemm_f32_gpu.py tests/test_dtypes_gpu.py > gpurun_out/r6n_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r6n_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/gemm_f32_bench.py > gpurun_out/r6n_f32_bench.log 2>&1 || { tail -5 gpurun_out/r6n_f32_bench.log; exit 1; }
cat gpurun_out/r6n_f32_bench.log
