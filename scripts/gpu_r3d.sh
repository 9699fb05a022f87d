#!/bin/bash
# activation checkpointing: GPU tests, overhead at seq 2048, long-context reach (seq 32k / 64k)
export TMPDIR=/tmp
mkdir -p gpurun_out
S=scripts/gpu_check.sh
$S actest 400 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread -k "xent or activation" || exit 1
$S ac_2k_off 400 python bench.py --steps 6 --warmup 2 || exit 1
$S ac_2k_on 400 python bench.py --steps 6 --warmup 2 --activation-checkpointing -1 || exit 1
$S ac_32k_on 500 python bench.py --seq-len 32768 --steps 2 --warmup 1 --activation-checkpointing -1 || exit 1
$S ac_64k_on 700 python bench.py --seq-len 65536 --steps 2 --warmup 1 --activation-checkpointing -1 || exit 1
