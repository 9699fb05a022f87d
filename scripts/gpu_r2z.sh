#!/bin/bash
export TMPDIR=/tmp
mkdir -p gpurun_out
S=scripts/gpu_check.sh
for v in 0 1 2; do FT_FLASH_IGLP=$v $S fb_iglp$v 300 python -u scripts/flash_bench.py || exit 1; done
FT_FLASH_IGLP=1 $S flashtest1 600 python -u -m pytest tests/test_flash_attn_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread || exit 1
FT_FLASH_IGLP=2 $S flashtest2 600 python -u -m pytest tests/test_flash_attn_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread || exit 1
