#!/bin/bash
# Selective activation checkpointing A/B on Llama-3-8B long context: kept attention output
# (default) vs full block recompute (--recompute-attention), plus the bitwise GPU test.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/sac
C="bash scripts/gpu_check.sh"
$C sac/test 300 python -u -m pytest tests/test_kernels_gpu.py -k activation_checkpointing -x -v --timeout 200 --timeout-method thread || exit $?
grep -q "passed" gpurun_out/sac/test.log && ! grep -q "failed" gpurun_out/sac/test.log || exit 1
B="python bench.py --model llama3-8b --no-ckpt --activation-checkpointing -1"
$C sac/s32768_keep 300 $B --seq-len 32768 --steps 3 --warmup 1 || exit $?
$C sac/s32768_recompute 300 $B --seq-len 32768 --steps 3 --warmup 1 --recompute-attention || exit $?
$C sac/s65536_keep 300 $B --seq-len 65536 --steps 2 --warmup 1 || exit $?
$C sac/s32768_half_keep 300 python bench.py --model llama3-8b --no-ckpt --activation-checkpointing 16 --seq-len 32768 --steps 3 --warmup 1 || exit $?
