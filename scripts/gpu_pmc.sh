#!/bin/bash
# counter list + PMC counters of the flash kernels (each pass its own run, kernel-trace only)
export TMPDIR=/tmp
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pmc
timeout -k 10 120 rocprofv3 -L > gpurun_out/pmc/avail.txt 2>&1
echo "list rc=$?"
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES SQ_WAVE_CYCLES -d gpurun_out/pmc/a -o run --output-format csv -- python3 scripts/flash_bench.py > gpurun_out/pmc/a.log 2>&1
echo "pmc rc=$?"
