#!/bin/bash
# fp16 / fp32 model dtypes on one MI355X: the dtype test file, then the bf16 kernel suites
# (regression check of the templated kernels). Stops at the first failing step.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_dtypes_gpu.py -x -v --timeout 200 --timeout-method thread > gpurun_out/dtypes.log 2>&1 || { tail -40 gpurun_out/dtypes.log; exit 1; }
tail -1 gpurun_out/dtypes.log
timeout -k 10 500 python -u -m pytest tests/test_kernels_gpu.py tests/test_flash_attn_gpu.py tests/test_gemm_gpu.py tests/test_head_xent_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/kern.log 2>&1 || { tail -30 gpurun_out/kern.log; exit 1; }
tail -1 gpurun_out/kern.log
