#!/bin/bash
export TMPDIR=/tmp
mkdir -p gpurun_out
S=scripts/gpu_check.sh
$S graph_tiny 300 python scripts/graph_probe.py tiny || exit 1
$S graph_g2s 300 python scripts/graph_probe.py gpt2-small || exit 1
$S graph_g2m 300 python scripts/graph_probe.py gpt2-medium || exit 1
