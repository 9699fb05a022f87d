#!/bin/bash
export TMPDIR=/tmp
mkdir -p gpurun_out
S=scripts/gpu_check.sh
$S mem_2k 300 python scripts/mem_probe.py --seq-len 2048 || exit 1
$S mem_16k 400 python scripts/mem_probe.py --seq-len 16384 --steps 3 || exit 1
$S mem_32k_rc 400 python scripts/mem_probe.py --seq-len 32768 --recompute -1 --steps 3 || exit 1
