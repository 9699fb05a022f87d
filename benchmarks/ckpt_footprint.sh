#!/bin/bash
# Checkpoint save vs HBM footprint (BASELINE config 5), run on the GPU box: writer throughput of the box's disk, then the 8B
# save in both snapshot modes at seq 2048 (~71 GB in use) and seq 32768 with block recompute (~105 GB).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; L=gpurun_out/ckpt_footprint.log; rm -f $L
df -T /tmp >> $L 2>&1
timeout -k 10 300 python3 scripts/ckpt_write_bench.py >> $L 2>&1 || exit $?
for args in "--ckpt-mode hbm" "--ckpt-mode host" "--seq-len 32768 --activation-checkpointing -1 --ckpt-mode auto" "--seq-len 32768 --activation-checkpointing -1 --ckpt-mode host"; do
  out=$(timeout -k 10 400 python3 bench.py --steps 5 --warmup 2 $args 2>/dev/null) || exit $?
  echo "== bench $args" >> $L
  echo "$out" | python3 -c "import json,sys; j=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(json.dumps({k: j[k] for k in ('ms_per_step','tokens_per_s_per_gpu','hbm_peak_gb','ckpt_save')}))" >> $L || exit $?
done
