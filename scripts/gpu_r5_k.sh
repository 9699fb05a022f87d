#!/bin/bash
# Round 5, session K: grouped tile raster — tests + per-product A/B.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gemm_w4t_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r5k_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r5k_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u scripts/w4_raster_bench.py ${GS:-0 2 4 8} > gpurun_out/r5k_raster.log 2>&1; rc=$?
cat gpurun_out/r5k_raster.log; exit $rc
