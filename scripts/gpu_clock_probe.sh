#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/clk
timeout -s KILL 200 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE -d gpurun_out/clk/step -o run --output-format csv -- python3 bench.py --steps 4 --warmup 2 --no-ckpt > gpurun_out/clk/step.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE -d gpurun_out/clk/iso -o run --output-format csv -- python3 scripts/gemm_pmc_probe.py > gpurun_out/clk/iso.log 2>&1 || exit 1
echo ok
