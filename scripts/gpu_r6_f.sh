#!/bin/bash
# Round 6, session F: w4 numerics after the epilogue split, then the safe 8B preempt chain.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gemm_w4t_gpu.py tests/test_gemm_gpu.py tests/test_w4_paths_gpu.py > gpurun_out/r6f_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r6f_tests.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_ft_logs_r6.sh
