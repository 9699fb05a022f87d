#!/bin/bash
# Round 5, session H: forward key halves — tests, timeline, bench.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_flash_attn_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r5h_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r5h_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u scripts/flash_fwd_timeline.py > gpurun_out/r5h_tl_b1.log 2>&1 &&
timeout -k 10 120 python -u scripts/flash_fwd_timeline.py 8192 32 8 128 > gpurun_out/r5h_tl_s8k.log 2>&1 &&
timeout -k 10 120 python -u scripts/flash_bench.py > gpurun_out/r5h_flash_b1.log 2>&1 &&
timeout -k 10 120 python -u scripts/flash_bench.py 2048 32 8 128 4 > gpurun_out/r5h_flash_b4.log 2>&1
rc=$?; cat gpurun_out/r5h_tl_b1.log; head -3 gpurun_out/r5h_flash_b*.log; exit $rc
