#!/bin/bash
# Same-box A/B of two kernel-library builds (FT_KERNELS_SO): abtest/_kernels_prev.so vs the tree's.
#   bash scripts/so_ab.sh <tag>
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
tag=$1
PREV=$GRAFT_REPO_ROOT/abtest/_kernels_prev.so
timeout -k 10 400 python -u -m pytest tests/test_gemm_w4t_gpu.py tests/test_gemm_gpu.py -q --maxfail 3 --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/${tag}_tests.log 2>&1; rc=$?
tail -2 gpurun_out/${tag}_tests.log
[ $rc -eq 0 ] || exit $rc
for v in prev cur prev cur; do
  if [ $v = prev ]; then export FT_KERNELS_SO=$PREV; else unset FT_KERNELS_SO; fi
  timeout -k 10 300 python -u scripts/w4_split_bench.py > gpurun_out/${tag}_split_$v.log 2>&1 || exit 1
  timeout -k 10 300 python -u scripts/gemm_w4t_bench.py > gpurun_out/${tag}_w4t_$v.log 2>&1 || exit 1
done
for v in prev cur prev cur; do
  if [ $v = prev ]; then export FT_KERNELS_SO=$PREV; else unset FT_KERNELS_SO; fi
  timeout -k 10 300 python -u bench.py --steps 12 --warmup 3 --no-ckpt > gpurun_out/${tag}_bench_$v.log 2>&1 || exit 1
  echo "$v $(tail -1 gpurun_out/${tag}_bench_$v.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["sclk_mhz_p50"], d["power_w_p50"])')" | tee -a gpurun_out/${tag}_bench_summary.log
done
