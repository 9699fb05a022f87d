#!/bin/bash
# Round 6, session AD: per-kernel times of the 3- and 4-kernel GQA flash backward (kernel trace).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
for v in 1 0; do
  rm -rf gpurun_out/r6ad_p$v
  FOLD3_ONLY=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r6ad_p$v -o run --output-format csv -- python3 scripts/flash_fold3_ab.py > gpurun_out/r6ad_p$v.log 2>&1 || exit 1
  echo "## fold3=$v"; python3 - <<PY
import csv, glob
f = glob.glob("gpurun_out/r6ad_p$v/**/run_kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if "flash" in r["Name"]:
        print(f"{float(r['AverageNs'])/1e3:8.1f} us  {int(r['Calls']):5d}  {r['Name'][:90]}")
PY
  rm -rf gpurun_out/r6ad_p$v
done
