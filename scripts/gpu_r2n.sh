#!/bin/bash
export TMPDIR=/tmp
mkdir -p gpurun_out
S=scripts/gpu_check.sh
$S graph_small 300 python -u scripts/graph_probe.py gpt2-small || exit 1
$S graph_medium 300 python -u scripts/graph_probe.py gpt2-medium || exit 1
