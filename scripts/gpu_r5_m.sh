#!/bin/bash
# Round 5, session M: GPU suite at HEAD, then a kernel-trace profile of the 8B bench.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --maxfail 5 --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r5m_gpu_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r5m_gpu_tests.log
[ $rc -eq 0 ] || exit $rc
rm -rf gpurun_out/prof_m && mkdir -p gpurun_out/prof_m
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_m -o run --output-format csv -- python3 bench.py --steps 5 --warmup 3 --no-ckpt > gpurun_out/r5m_prof.log 2>&1; rc=$?
tail -1 gpurun_out/r5m_prof.log | cut -c1-200
find gpurun_out/prof_m -name "*stats*" | head -3
exit $rc
