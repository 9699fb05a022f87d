#!/bin/bash
# Round 5, session I: probes (flash / w4 timing) tests + the w4 timeline.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_flash_attn_gpu.py tests/test_gemm_w4t_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r5i_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r5i_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/w4_timeline.py > gpurun_out/r5i_w4_timeline.log 2>&1; rc=$?
cat gpurun_out/r5i_w4_timeline.log; exit $rc
