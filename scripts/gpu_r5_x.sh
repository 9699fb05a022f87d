#!/bin/bash
# Round 5, session X: PMC passes over the grouped-raster probe (each pass its own run, kernel-trace only).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/pmc_raster
i=0
for set in "TCC_HIT_sum TCC_MISS_sum SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" "FETCH_SIZE" "SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAVE_CYCLES"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $set -d gpurun_out/pmc_raster/p$i -o run --output-format csv -- python3 scripts/w4_raster_pmc_probe.py > gpurun_out/pmc_raster/p$i.log 2>&1 || { echo "pass $i rc=$?"; tail -3 gpurun_out/pmc_raster/p$i.log; exit 1; }
done
python3 scripts/w4_raster_pmc_probe.py --summary gpurun_out/pmc_raster > gpurun_out/r5x_raster_pmc.txt && cat gpurun_out/r5x_raster_pmc.txt
