#!/bin/bash
# Hardware rcp/sqrt in AdamW / SwiGLU: numerics tests, power/clock of AdamW alone and beside the
# GEMM chain, and the same-process 8B step A/B.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "adamw or swiglu or optim or train or model" > gpurun_out/fm_tests.log 2>&1 || { tail -30 gpurun_out/fm_tests.log; exit 1; }
tail -1 gpurun_out/fm_tests.log
timeout -k 10 300 python scripts/power_probe.py 2>&1 | grep -v "amdgpu.ids\|^hwmon" | tee gpurun_out/fm_power.log || exit 1
timeout -k 10 400 python scripts/ab_step.py --knobs fastmath --rounds 4 --steps 8 2>&1 | grep "\[ab\]" | tee gpurun_out/fm_ab.log || exit 1
