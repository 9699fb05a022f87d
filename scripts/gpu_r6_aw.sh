#!/bin/bash
# Round 6, session AW: full GPU suite + smoke + bench (no arguments) at HEAD, and an fp32 train.py run
# (the product loop with the fp32 MFMA GEMM, its startup log line).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --maxfail 5 --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r6aw_gpu_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r6aw_gpu_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6aw_smoke.log 2>&1 || exit 1
tail -1 gpurun_out/r6aw_smoke.log
timeout -k 10 400 python -u bench.py > gpurun_out/r6aw_bench_noargs.log 2>&1 || exit 1
tail -1 gpurun_out/r6aw_bench_noargs.log | cut -c1-400
rm -rf /tmp/ftf32 && mkdir -p /tmp/ftf32
SLURM_JOB_ID=6100 timeout -k 10 300 python -u train.py --model gpt2-small --synthetic-data --vocab-size 50304 --sequence-length 2048 \
  --batch-size 1 --model-dtype fp32 --training-steps 60 --logging-frequency 10 --checkpoint-path /tmp/ftf32 > gpurun_out/r6aw_train_fp32.log 2>&1 || { tail -5 gpurun_out/r6aw_train_fp32.log; exit 1; }
grep -E "model-dtype fp32|Training step: (10|30|50|60) |Training completed" gpurun_out/r6aw_train_fp32.log | cut -c1-250
