#!/bin/bash
export TMPDIR=/tmp
mkdir -p gpurun_out
S=scripts/gpu_check.sh
$S bench 600 python bench.py || exit 1
$S bench2 600 python bench.py || exit 1
$S bench_s4096 600 python bench.py --seq-len 4096 --steps 6 --warmup 2 || exit 1
$S bench_s16384 600 python bench.py --seq-len 16384 --steps 3 --warmup 1 || exit 1
