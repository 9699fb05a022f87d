#!/bin/bash
# stream-ordered dW operand lifetime (no record_stream): tests, HBM reserve, benches
export TMPDIR=/tmp
mkdir -p gpurun_out
S=scripts/gpu_check.sh
$S pk_test 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_ft_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread || exit 1
$S pk_fr_2k 300 python scripts/mem_probe.py --free-run --steps 6 || exit 1
$S pk_fr_16k 400 python scripts/mem_probe.py --free-run --steps 4 --seq-len 16384 || exit 1
$S pk_2k 300 python bench.py || exit 1
FT_DW_LAG=8 $S pk_2k_l8 300 python bench.py || exit 1
FT_DW_LAG=2 $S pk_2k_l2 300 python bench.py || exit 1
$S pk_2k2 300 python bench.py || exit 1
$S pk_16k 400 python bench.py --seq-len 16384 --steps 3 --warmup 2 || exit 1
$S pk_32k 500 python bench.py --seq-len 32768 --steps 3 --warmup 2 --activation-checkpointing -1 || exit 1
PYTORCH_HIP_ALLOC_CONF=max_split_size_mb:512 $S pk_32k_m 500 python bench.py --seq-len 32768 --steps 3 --warmup 2 --activation-checkpointing -1 || exit 1
