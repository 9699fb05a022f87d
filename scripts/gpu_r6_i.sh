#!/bin/bash
# Round 6, session I: re-run the tests that failed in session G (twice for the DP graph file).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
for r in 1 2; do
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_dp_rccl_gpu.py tests/test_kernels_gpu.py tests/test_graphs_gpu.py > gpurun_out/r6i_tests_$r.log 2>&1
rc=$?; tail -3 gpurun_out/r6i_tests_$r.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
done
