#!/bin/bash
# Round 5, session B: full GPU suite, 8B bench, GPT-2 presets (vocab 50304 / 131072) after the
# routing cleanup (w4 split-K routes for the GPT-2 head dX and the wide projections).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q --maxfail 5 --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r5_gpu_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r5_gpu_tests.log
# assertion failures (rc 1) still let the benches run; a timeout / crash ends the session
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-ckpt > gpurun_out/r5_bench_b.log 2>&1 || exit 1
tail -1 gpurun_out/r5_bench_b.log | cut -c1-400
: > gpurun_out/r5_gpt2_bench_b.jsonl
for m in gpt2-small gpt2-medium; do
  for v in 50304 131072; do
    timeout -k 10 200 python -u bench.py --model $m --graph --vocab-size $v --steps 30 --warmup 5 --no-ckpt > gpurun_out/gb_${m}_$v.log 2>&1 || { tail -5 gpurun_out/gb_${m}_$v.log; exit 1; }
    tail -1 gpurun_out/gb_${m}_$v.log >> gpurun_out/r5_gpt2_bench_b.jsonl
  done
done
echo "gpt2 ok"
timeout -k 10 300 python -u scripts/w4_overhead_probe.py > gpurun_out/r5_w4_overhead.log 2>&1 || exit 1
echo "probe ok"
