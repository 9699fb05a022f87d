#!/bin/bash
# Round 5, session Y: L2 behaviour of the flash kernels at the 8B layer (PMC, kernel-trace only).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/pmc_flash
i=0
for set in "TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE" "FETCH_SIZE"; do
  i=$((i+1))
  timeout -s KILL 180 rocprofv3 --kernel-trace --pmc $set -d gpurun_out/pmc_flash/p$i -o run --output-format csv -- python3 scripts/flash_bench.py > gpurun_out/pmc_flash/p$i.log 2>&1 || { echo "pass $i rc=$?"; tail -3 gpurun_out/pmc_flash/p$i.log; exit 1; }
done
python3 scripts/pmc_summary.py gpurun_out/pmc_flash > gpurun_out/r5y_flash_pmc.txt && cat gpurun_out/r5y_flash_pmc.txt
