#!/bin/bash
# flash attention: numerics, timing, per-kernel stats
export TMPDIR=/tmp
mkdir -p gpurun_out
S=scripts/gpu_check.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
$S flash_tests 400 python -m pytest tests/test_flash_attn_gpu.py -x -q || exit 1
$S flash_bench 300 python scripts/flash_bench.py || exit 1
$S flash_prof 400 rocprofv3 --kernel-trace --stats -d gpurun_out/flash_prof -o run --output-format csv -- python3 scripts/flash_bench.py || exit 1
