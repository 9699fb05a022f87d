#!/bin/bash
# Round 5, session L: grouped raster by default — w4 tests, same-box step A/B, bench.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gemm_w4t_gpu.py tests/test_w4_paths_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r5l_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r5l_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u scripts/ab_step.py --knobs raster --rounds 3 > gpurun_out/r5l_ab_raster.log 2>&1 || exit 1
grep "best" gpurun_out/r5l_ab_raster.log
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r5l_bench.log 2>&1 || exit 1
tail -1 gpurun_out/r5l_bench.log | cut -c1-400
