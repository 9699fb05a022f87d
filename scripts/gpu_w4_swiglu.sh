#!/bin/bash
# w1|w3 GEMM with the SwiGLU epilogue: numerics tests, model-level GPU tests, then the 8B step A/B.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gemm_gpu.py tests/test_graphs_gpu.py tests/test_dtypes_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/swiglu_tests.log 2>&1 || { tail -30 gpurun_out/swiglu_tests.log; exit 1; }
tail -1 gpurun_out/swiglu_tests.log
timeout -k 10 600 python scripts/ab_step.py --knobs w4swiglu --rounds 4 --steps 8 2>&1 | grep "\[ab\]" | tee gpurun_out/ab_w4swiglu.log || exit 1
