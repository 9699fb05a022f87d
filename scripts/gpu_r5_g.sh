#!/bin/bash
# Round 5, session G: flash fwd/bwd scaling with batch (tail vs loop efficiency) + per-phase clock.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 120 python -u scripts/flash_bench.py > gpurun_out/r5g_flash_b1.log 2>&1 &&
timeout -k 10 120 python -u scripts/flash_bench.py 2048 32 8 128 4 > gpurun_out/r5g_flash_b4.log 2>&1 &&
timeout -k 10 120 python -u scripts/flash_bench.py 8192 32 8 128 1 > gpurun_out/r5g_flash_s8k.log 2>&1 &&
timeout -k 10 300 python -u scripts/phase_clock.py 30 > gpurun_out/r5g_phase_clock.log 2>&1
rc=$?; head -4 gpurun_out/r5g_flash_b*.log gpurun_out/r5g_flash_s8k.log; cat gpurun_out/r5g_phase_clock.log; exit $rc
