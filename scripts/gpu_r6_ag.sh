#!/bin/bash
# Round 6, session AG: the optimizer's gating unit on one GPU (--bucket-mb: AdamW launch size and the
# forward's per-layer waits), 8B bench, alternating.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
for v in 64 256 32 64 256 32; do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-ckpt --bucket-mb $v > gpurun_out/r6ag_b.json 2>gpurun_out/r6ag_b.err || { tail -3 gpurun_out/r6ag_b.err; exit 1; }
  echo "bucket_mb=$v $(python3 -c "import json;d=json.loads(open('gpurun_out/r6ag_b.json').read().strip().splitlines()[-1]);print(d['ms_per_step'], d.get('sclk_mhz_p50'), d.get('buckets'))")" >> gpurun_out/r6ag_bench.log
done
cat gpurun_out/r6ag_bench.log
