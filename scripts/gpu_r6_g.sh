#!/bin/bash
# Round 6, session G: the full GPU suite + smoke, then 8B bench A/B round-5 tree vs HEAD (x3).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -q --maxfail 5 --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r6g_gpu_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r6g_gpu_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6g_smoke.log 2>&1 || exit 1
tail -1 gpurun_out/r6g_smoke.log
j() { python -c "import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); print(d['ms_per_step'], d.get('sclk_mhz_p50'), d.get('power_w_p50'))"; }
for r in 1 2 3; do for v in r5 head; do
  if [ $v = r5 ]; then cd $R/abtree_r5; else cd $R; fi
  timeout -k 10 300 python -u bench.py --steps 15 --warmup 4 --no-ckpt > $R/gpurun_out/r6g_8b_${v}_$r.log 2>&1 || exit 1
  echo "8b $v $r $(j $R/gpurun_out/r6g_8b_${v}_$r.log)"
done; done
