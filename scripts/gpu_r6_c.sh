#!/bin/bash
# Round 6, session C: ZeRO-1 under the HIP graph (single-stream collectives), graph-mode fault
# routing and the peer-loss solo save, split-K lost-hand-off path + dW split / M tail, graph == eager.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
P=scripts/capture_collectives_probe.py
timeout -k 10 600 python -u $P > gpurun_out/r6c_capture_probe.log 2>&1
grep -E "^=== " gpurun_out/r6c_capture_probe.log
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_dp_rccl_gpu.py tests/test_graphs_gpu.py tests/test_gemm_w4t_gpu.py tests/test_gemm_gpu.py > gpurun_out/r6c_tests.log 2>&1
rc=$?; grep -E "passed|failed|FAILED|ERROR" gpurun_out/r6c_tests.log | tail -15; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-ckpt > gpurun_out/r6c_bench.log 2>&1 || exit 1
tail -1 gpurun_out/r6c_bench.log | cut -c1-250
timeout -k 10 300 python -u scripts/gpt2_gemm_probe.py > gpurun_out/r6c_gpt2_probe_small.log 2>&1 || exit 1
timeout -k 10 300 python -u scripts/gpt2_gemm_probe.py 1024 2816 3072 > gpurun_out/r6c_gpt2_probe_medium.log 2>&1 || exit 1
cut -c1-140 gpurun_out/r6c_gpt2_probe_small.log gpurun_out/r6c_gpt2_probe_medium.log
for m in gpt2-small gpt2-medium; do for w in 0 1; do
  FT_W4_SMALL=$w timeout -k 10 300 python -u bench.py --model $m --vocab-size 50304 --graph --steps 50 --warmup 5 --no-ckpt > gpurun_out/r6c_${m}_w4small$w.log 2>&1 || exit 1
  echo "$m FT_W4_SMALL=$w $(python -c "import json,sys; d=json.loads(open('gpurun_out/r6c_${m}_w4small$w.log').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['mfu_vs_2.5PF_dense'], d.get('sclk_mhz_p50'))")"
done; done
