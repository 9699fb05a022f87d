#!/bin/bash
export TMPDIR=/tmp
mkdir -p gpurun_out
scripts/gpu_check.sh bw_bench 300 python scripts/bw_bench.py || exit 1
