#!/bin/bash
# Round 5, session C: persistent w4 grid -- its tests, the per-tile overhead probe, the 8B split /
# dW product bench, the step A/B and the bench.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gemm_w4t_gpu.py tests/test_gemm_gpu.py -q --maxfail 3 --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r5c_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r5c_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/w4_overhead_probe.py > gpurun_out/r5c_overhead.log 2>&1 && W4_PROBE_PERSIST=0 timeout -k 10 300 python -u scripts/w4_overhead_probe.py > gpurun_out/r5c_overhead_off.log 2>&1 || exit 1
timeout -k 10 300 python -u scripts/gemm_w4t_bench.py > gpurun_out/r5c_w4t_bench.log 2>&1 || exit 1
timeout -k 10 400 python -u scripts/ab_step.py --knobs persist --rounds 3 > gpurun_out/r5c_ab_persist.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-ckpt > gpurun_out/r5c_bench.log 2>&1 || exit 1
echo done
