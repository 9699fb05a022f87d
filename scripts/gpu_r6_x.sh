#!/bin/bash
# Round 6, session X: the LDS-DMA fp32 GEMM: numerics, DMA vs register form vs hipBLASLt on the
# products, fp32 step A/B.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_gemm_f32_gpu.py > gpurun_out/r6x_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r6x_tests.log; [ $rc -eq 0 ] || exit $rc
for v in 1 0; do
  echo "## dma=$v" >> gpurun_out/r6x_f32_bench.log
  timeout -k 10 300 python -u scripts/gemm_f32_bench.py --dma $v 2>&1 | grep -v amdgpu.ids >> gpurun_out/r6x_f32_bench.log || exit 1
done
cat gpurun_out/r6x_f32_bench.log
for m in gpt2-small; do
  timeout -k 10 400 python -u scripts/ab_step.py --model $m --vocab-size 50304 --dtype fp32 --knobs f32mfma \
    --rounds 4 --steps 10 > gpurun_out/r6x_ab_f32_$m.log 2>&1 || { tail -5 gpurun_out/r6x_ab_f32_$m.log; exit 1; }
  grep "best" gpurun_out/r6x_ab_f32_$m.log
done
