#!/bin/bash
# Round 6, session T: fp32 GEMM with the prefetch loads pinned at the loop top (sched_barrier):
# numerics of both forms, the persistent BK = 64 form vs the two-per-CU BK = 32 form vs hipBLASLt,
# fp32 step A/B.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_gemm_f32_gpu.py > gpurun_out/r6t_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r6t_tests.log; [ $rc -eq 0 ] || exit $rc
for v in 1 0; do
  echo "## persistent=$v" >> gpurun_out/r6t_f32_bench.log
  timeout -k 10 300 python -u scripts/gemm_f32_bench.py --persistent $v >> gpurun_out/r6t_f32_bench.log 2>&1 || { tail -5 gpurun_out/r6t_f32_bench.log; exit 1; }
done
grep -v amdgpu.ids gpurun_out/r6t_f32_bench.log
