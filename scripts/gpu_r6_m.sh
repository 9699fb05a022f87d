#!/bin/bash
# Round 6, session M: the conflict-free epilogue staging writes (8-B halves swapped in rows with
# bit 3 set): numerics of every epilogue form, LDS bank-conflict PMC pass per product, HEAD vs
# new on the 8B products and a same-box 8B bench.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r6m_pmc gpurun_out/r6m_pmc_head
timeout -k 10 400 python -u -m pytest -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_gemm_w4t_gpu.py tests/test_gemm_gpu.py tests/test_w4_paths_gpu.py tests/test_dtypes_gpu.py \
  > gpurun_out/r6m_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r6m_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_WAVES \
  -d gpurun_out/r6m_pmc -o run --output-format csv -- python3 scripts/w4_epi_pmc_probe.py > gpurun_out/r6m_pmc.log 2>&1 || { echo "pmc rc=$?"; tail -3 gpurun_out/r6m_pmc.log; exit 1; }
(cd abtree_r5 && timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_WAVES \
  -d ../gpurun_out/r6m_pmc_head -o run --output-format csv -- python3 ../scripts/w4_epi_pmc_probe.py) > gpurun_out/r6m_pmc_head.log 2>&1 || { echo "pmc head rc=$?"; tail -3 gpurun_out/r6m_pmc_head.log; exit 1; }
{ echo "## HEAD (46f5b90)"; python3 scripts/w4_epi_pmc_probe.py --summary gpurun_out/r6m_pmc_head;
  echo "## swapped halves"; python3 scripts/w4_epi_pmc_probe.py --summary gpurun_out/r6m_pmc; } > gpurun_out/r6m_pmc_summary.txt
cat gpurun_out/r6m_pmc_summary.txt
for t in head new head new; do
  if [ $t = head ]; then d=abtree_r5; else d=.; fi
  echo "## $t" >> gpurun_out/r6m_w4t.log
  (cd $d && timeout -k 10 300 python -u scripts/gemm_w4t_bench.py) >> gpurun_out/r6m_w4t.log 2>&1 || exit 1
done
for t in head new head new; do
  if [ $t = head ]; then d=abtree_r5; else d=.; fi
  (cd $d && timeout -k 10 300 python -u bench.py --steps 20 --warmup 5) > gpurun_out/r6m_bench_$t.json 2>gpurun_out/r6m_bench_$t.err || exit 1
  echo "$t $(cat gpurun_out/r6m_bench_$t.json)" >> gpurun_out/r6m_bench.log
done
cat gpurun_out/r6m_bench.log
