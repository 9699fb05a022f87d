#!/bin/bash
# Round 6, session AR: long-context 8B throughput refresh (seq 4096 / 16384; 32768 with blocks recomputed).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
for S in 4096 16384; do
  timeout -k 10 240 python bench.py --seq-len $S --steps 8 --warmup 3 --no-ckpt > gpurun_out/r6ar_s$S.log 2>&1 || { tail -5 gpurun_out/r6ar_s$S.log; exit 1; }
  echo "seq $S $(python3 -c "import json;d=json.loads(open('gpurun_out/r6ar_s$S.log').read().strip().splitlines()[-1]);print(d['value'], 'tok/s', d['ms_per_step'], 'ms', d.get('sclk_mhz_p50'), 'MHz', d.get('hbm_peak_gb'), 'GB')")"
done
timeout -k 10 300 python bench.py --seq-len 32768 --activation-checkpointing -1 --steps 5 --warmup 2 --no-ckpt > gpurun_out/r6ar_s32768.log 2>&1 || { tail -5 gpurun_out/r6ar_s32768.log; exit 1; }
echo "seq 32768 recompute $(python3 -c "import json;d=json.loads(open('gpurun_out/r6ar_s32768.log').read().strip().splitlines()[-1]);print(d['value'], 'tok/s', d['ms_per_step'], 'ms', d.get('sclk_mhz_p50'), 'MHz', d.get('hbm_peak_gb'), 'GB')")"
