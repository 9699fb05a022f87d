#!/bin/bash
# Pipelined flash forward: numerics tests, then timings at the 8B layer shape and long context.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_flash_attn_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/flash_tests.log 2>&1 || { tail -30 gpurun_out/flash_tests.log; exit 1; }
tail -2 gpurun_out/flash_tests.log
for shape in "2048 32 8 128" "8192 32 8 128" "2048 12 12 64" "2048 16 16 64"; do
  timeout -k 10 120 python scripts/flash_bench.py $shape 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/flash_bench.log || exit 1
done
