#!/bin/bash
# Round 6, session L: the dW round-remainder split (FT_W4_REMAINDER): numerics, the qkv dW alone,
# same-process 8B step A/B.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_gemm_w4t_gpu.py -k "remainder or dead_tail or dw_split" > gpurun_out/r6l_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r6l_tests.log; [ $rc -eq 0 ] || exit $rc
for v in 0 1; do FT_W4_REMAINDER=$v timeout -k 10 300 python -u scripts/gemm_w4t_bench.py > gpurun_out/r6l_w4t_rem$v.log 2>&1 || exit 1; done
grep "qkv dW" gpurun_out/r6l_w4t_rem0.log gpurun_out/r6l_w4t_rem1.log
timeout -k 10 600 python -u scripts/ab_step.py --knobs remainder --rounds 4 --steps 10 > gpurun_out/r6l_ab_remainder.log 2>&1 || exit 1
grep "best" gpurun_out/r6l_ab_remainder.log
