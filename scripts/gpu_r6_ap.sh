#!/bin/bash
# Round 6, session AP: thread-local graph capture (the RCCL watchdog's event queries during capture):
# the DP graph tests, three passes, and the graph tests.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
for i in 1 2 3; do
  timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    tests/test_dp_rccl_gpu.py tests/test_graphs_gpu.py > gpurun_out/r6ap_tests_$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc $(tail -1 gpurun_out/r6ap_tests_$i.log)"
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
done
