#!/bin/bash
# Board power / clock during the real 8B step, and flash fwd/bwd at B=1 vs B=4 (causal imbalance).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 200 python scripts/power_step.py 5 2>&1 | grep -v amdgpu.ids | tee gpurun_out/power_step.log || exit 1
timeout -k 10 200 python scripts/power_probe.py 2>&1 | grep -v "amdgpu.ids\|^hwmon" | tee -a gpurun_out/power_step.log || exit 1
for b in 1 4; do
  timeout -k 10 120 python scripts/flash_bench.py 2048 32 8 128 $b 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/flash_b.log || exit 1
done
