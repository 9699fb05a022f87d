#!/bin/bash
# Round 5, session S: same-box A/B of the round-4 final tree (abtree_r4, commit 84aa2f6) vs HEAD, bench.py alternated.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
for v in r4 head r4 head r4 head; do
  if [ $v = r4 ]; then d=$GRAFT_REPO_ROOT/abtree_r4; else d=$GRAFT_REPO_ROOT; fi
  (cd $d && timeout -k 10 300 python -u bench.py --steps 15 --warmup 4 --no-ckpt) > gpurun_out/r5s_bench_$v.log 2>&1 || exit 1
  echo "$v $(tail -1 gpurun_out/r5s_bench_$v.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d.get("sclk_mhz_p50"), d.get("power_w_p50"))')" | tee -a gpurun_out/r5s_ab_summary.log
done
