#!/bin/bash
# w4 GEMM: GPU tests (gemm + model), isolated bench, then the step-level A/B of the fused
# QKV+RoPE projection and of every forward GEMM on the kernel.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/w4_tests.log 2>&1 || { tail -30 gpurun_out/w4_tests.log; exit 1; }
tail -2 gpurun_out/w4_tests.log
timeout -k 10 300 python -u scripts/gemm_w4_bench.py --rounds 3 > gpurun_out/w4_bench.log 2>&1 || { tail -10 gpurun_out/w4_bench.log; exit 1; }
tail -10 gpurun_out/w4_bench.log
timeout -k 10 500 python -u scripts/ab_step.py --knobs w4fwd,w4dw --rounds 3 --steps 6 > gpurun_out/w4_ab.log 2>&1 || { tail -5 gpurun_out/w4_ab.log; exit 1; }
tail -5 gpurun_out/w4_ab.log
