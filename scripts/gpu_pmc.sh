#!/bin/bash
# rocprofv3 PMC passes (each its own run, kernel-trace only) over a probe script.
#   bash scripts/gpu_pmc.sh <tag> <python script + args>
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tag=$1; shift
mkdir -p gpurun_out/pmc_$tag
i=0
for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE" \
           "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $set -d gpurun_out/pmc_$tag/p$i -o run --output-format csv -- python3 "$@" > gpurun_out/pmc_$tag/p$i.log 2>&1 || { echo "pass $i rc=$?"; exit 1; }
done
echo ok
