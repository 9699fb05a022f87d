#!/bin/bash
# Round 6, session J: w4 dead-tail DMAs through null descriptors (FT_W4_DEADZERO): numerics, product
# times with / without, same-process 8B step A/B, and bench.py alternated.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gemm_w4t_gpu.py tests/test_gemm_gpu.py tests/test_w4_paths_gpu.py > gpurun_out/r6j_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r6j_tests.log; [ $rc -eq 0 ] || exit $rc
for v in 0 1; do
  FT_W4_DEADZERO=$v timeout -k 10 300 python -u scripts/gemm_w4t_bench.py > gpurun_out/r6j_w4t_dz$v.log 2>&1 || exit 1
  FT_W4_DEADZERO=$v timeout -k 10 300 python -u scripts/w4_split_bench.py > gpurun_out/r6j_split_dz$v.log 2>&1 || exit 1
done
paste <(grep -E "dX|dW|fwd" gpurun_out/r6j_w4t_dz0.log | cut -c1-60) <(grep -E "dX|dW|fwd" gpurun_out/r6j_w4t_dz1.log | cut -c36-60)
timeout -k 10 600 python -u scripts/ab_step.py --knobs deadzero --rounds 4 --steps 10 > gpurun_out/r6j_ab_deadzero.log 2>&1 || exit 1
grep "best" gpurun_out/r6j_ab_deadzero.log
j() { python -c "import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); print(d['ms_per_step'], d.get('sclk_mhz_p50'), d.get('power_w_p50'))"; }
for r in 1 2; do for v in 0 1; do
  FT_W4_DEADZERO=$v timeout -k 10 300 python -u bench.py --steps 15 --warmup 4 --no-ckpt > gpurun_out/r6j_8b_dz${v}_$r.log 2>&1 || exit 1
  echo "8b deadzero=$v $r $(j gpurun_out/r6j_8b_dz${v}_$r.log)"
done; done
