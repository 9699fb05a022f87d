#!/bin/bash
# GPT-2 kernel breakdowns (rocprofv3, no checkpoint block) + flash head_dim-64 long-context check.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/prof_s gpurun_out/prof_m; mkdir -p gpurun_out/prof_s gpurun_out/prof_m
set -o pipefail
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_s -o run --output-format csv -- python3 bench.py --model gpt2-small --steps 10 --warmup 3 --no-ckpt > gpurun_out/prof_s.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_m -o run --output-format csv -- python3 bench.py --model gpt2-medium --steps 10 --warmup 3 --no-ckpt > gpurun_out/prof_m.log 2>&1 || exit $?
timeout -k 10 120 python3 scripts/flash_bench.py 8192 16 16 64 > gpurun_out/flash_d64.log 2>&1 || exit $?
timeout -k 10 120 python3 scripts/flash_bench.py 2048 12 12 64 >> gpurun_out/flash_d64.log 2>&1 || exit $?
timeout -k 10 300 python3 -u -m pytest tests/test_flash_attn_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/flash_test.log 2>&1 || exit $?
