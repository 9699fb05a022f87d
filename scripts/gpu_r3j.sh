#!/bin/bash
# side-stream buffers from the compute stream's pool: tests, HBM reserve, benches
export TMPDIR=/tmp
mkdir -p gpurun_out
S=scripts/gpu_check.sh
$S pj_test 500 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread || exit 1
$S pj_fr_2k 300 python scripts/mem_probe.py --free-run --steps 6 || exit 1
$S pj_fr_16k 400 python scripts/mem_probe.py --free-run --steps 4 --seq-len 16384 || exit 1
$S pj_2k 300 python bench.py || exit 1
$S pj_16k 400 python bench.py --seq-len 16384 --steps 3 --warmup 2 || exit 1
$S pj_32k 500 python bench.py --seq-len 32768 --steps 3 --warmup 2 --activation-checkpointing -1 || exit 1
PYTORCH_HIP_ALLOC_CONF=max_split_size_mb:512 $S pj_16k_m 400 python bench.py --seq-len 16384 --steps 3 --warmup 2 || exit 1
PYTORCH_HIP_ALLOC_CONF=max_split_size_mb:512 $S pj_32k_m 500 python bench.py --seq-len 32768 --steps 3 --warmup 2 --activation-checkpointing -1 || exit 1
$S pj_2k2 300 python bench.py || exit 1
