#!/bin/bash
# Round 5, session Z (final): the full GPU suite + smoke + bench at HEAD.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --maxfail 5 --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r5z_gpu_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r5z_gpu_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5z_smoke.log 2>&1 || exit 1
tail -1 gpurun_out/r5z_smoke.log
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r5z_bench.log 2>&1 || exit 1
tail -1 gpurun_out/r5z_bench.log | cut -c1-300
