#!/bin/bash
export TMPDIR=/tmp
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/kprof gpurun_out/kprof_old
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/kprof -o run --output-format csv -- python3 scripts/kernel_bw_bench.py > gpurun_out/kprof.log 2>&1 || exit 1
FT_KERNELS_SO=abso/_kernels_t13.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/kprof_old -o run --output-format csv -- python3 scripts/kernel_bw_bench.py > gpurun_out/kprof_old.log 2>&1 || exit 1
