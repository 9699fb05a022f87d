#!/bin/bash
# Round 5, session R: GPT-2 routing refinement — w4 path tests + GPT-2 benches at both vocabularies.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_w4_paths_gpu.py tests/test_kernels_gpu.py tests/test_gemm_gpu.py tests/test_graphs_gpu.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r5r_tests.log 2>&1; rc=$?
tail -2 gpurun_out/r5r_tests.log
[ $rc -eq 0 ] || exit $rc
for m in gpt2-small gpt2-medium; do for V in 50304 131072; do
  timeout -k 10 300 python -u bench.py --model $m --vocab-size $V --graph --steps 30 --warmup 5 --no-ckpt > gpurun_out/r5r_${m}_$V.log 2>&1 || exit 1
  tail -1 gpurun_out/r5r_${m}_$V.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["config"]["model"], '$V', d["ms_per_step"], d["mfu_vs_2.5PF_dense"], d.get("sclk_mhz_p50"))'
done; done
