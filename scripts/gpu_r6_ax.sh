#!/bin/bash
# Round 6, session AX: PMC pass of the LDS-DMA fp32 GEMM vs hipBLASLt on the 8B w1|w3 forward.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r6ax_pmc
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS GRBM_GUI_ACTIVE \
  -d gpurun_out/r6ax_pmc -o run --output-format csv -- python3 scripts/f32_pmc_probe.py > gpurun_out/r6ax_pmc.log 2>&1 || { echo "pmc rc=$?"; tail -3 gpurun_out/r6ax_pmc.log; exit 1; }
python3 scripts/f32_pmc_probe.py --summary gpurun_out/r6ax_pmc | tee gpurun_out/r6ax_pmc_summary.txt
rm -rf gpurun_out/r6ax_pmc
