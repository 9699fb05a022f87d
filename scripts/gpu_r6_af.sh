#!/bin/bash
# Round 6, session AF: the 8B bench step eager vs replayed as one HIP graph (--graph), alternating.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
for v in eager graph eager graph; do
  if [ $v = graph ]; then f=--graph; else f=; fi
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-ckpt $f > gpurun_out/r6af_b.json 2>gpurun_out/r6af_b.err || { tail -3 gpurun_out/r6af_b.err; exit 1; }
  echo "$v $(python3 -c "import json;d=json.loads(open('gpurun_out/r6af_b.json').read().strip().splitlines()[-1]);print(d['ms_per_step'], d.get('sclk_mhz_p50'), d.get('power_w_p50'), d.get('hbm_peak_gb'))")" >> gpurun_out/r6af_bench.log
done
cat gpurun_out/r6af_bench.log
