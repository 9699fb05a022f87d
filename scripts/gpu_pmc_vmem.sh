#!/bin/bash
# rocprofv3 PMC pass on the vector-memory issue path (kernel-trace only), over a probe script.
#   bash scripts/gpu_pmc_vmem.sh <tag> <python script + args>
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tag=$1; shift
mkdir -p gpurun_out/pmc_$tag
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc ${PMC:-SQ_INSTS_VMEM_RD SQ_INST_CYCLES_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES TA_BUSY_avr TA_BUFFER_READ_LDS_WAVEFRONTS_sum GRBM_GUI_ACTIVE} -d gpurun_out/pmc_$tag/p3 -o run --output-format csv -- python3 "$@" > gpurun_out/pmc_$tag/p3.log 2>&1 || { echo "pass rc=$?"; exit 1; }
echo ok
