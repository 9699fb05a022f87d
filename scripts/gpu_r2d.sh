#!/bin/bash
export TMPDIR=/tmp
mkdir -p gpurun_out
S=scripts/gpu_check.sh
$S gputests 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread || exit 1
$S ab_tonly 600 python -u scripts/ab_step.py --knobs tonly --rounds 3 --steps 8 || exit 1
$S bench 600 python bench.py || exit 1
