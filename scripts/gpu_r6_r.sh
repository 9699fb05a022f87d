#!/bin/bash
# Round 6, session R: fp32 GEMM -- LDS rows of 36 vs 40 floats (72 vs 80 KiB per workgroup) and a PMC
# pass against hipBLASLt on the 8B w1|w3 forward.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r6r_pmc
for v in sk40 sk36 sk40 sk36; do
  if [ $v = sk36 ]; then so=ablib/_kernels_sk36.so; else so=""; fi
  echo "## $v" >> gpurun_out/r6r_bench.log
  FT_KERNELS_SO=$so timeout -k 10 300 python -u scripts/gemm_f32_bench.py 2>&1 | grep llama3 >> gpurun_out/r6r_bench.log || exit 1
done
cat gpurun_out/r6r_bench.log
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS GRBM_GUI_ACTIVE \
  -d gpurun_out/r6r_pmc -o run --output-format csv -- python3 scripts/f32_pmc_probe.py > gpurun_out/r6r_pmc.log 2>&1 || { echo "pmc rc=$?"; tail -3 gpurun_out/r6r_pmc.log; exit 1; }
python3 scripts/f32_pmc_probe.py --summary gpurun_out/r6r_pmc | tee gpurun_out/r6r_pmc_summary.txt
