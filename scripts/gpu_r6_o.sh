#!/bin/bash
# Round 6, session O: fp32 MFMA GEMM (scratch-free prefetch, split-K for small grids): numerics +
# kernel vs hipBLASLt.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_gemm_f32_gpu.py tests/test_dtypes_gpu.py > gpurun_out/r6o_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r6o_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/gemm_f32_bench.py > gpurun_out/r6o_f32_bench.log 2>&1 || { tail -5 gpurun_out/r6o_f32_bench.log; exit 1; }
cat gpurun_out/r6o_f32_bench.log
