#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof_head
bash scripts/gpu_check.sh gputests 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit $?
grep -q "passed" gpurun_out/gputests.log && ! grep -q "failed" gpurun_out/gputests.log || exit 1
bash scripts/gpu_check.sh smoke 200 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
bash scripts/gpu_check.sh bench 400 python bench.py || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_head -o run --output-format csv -- python3 bench.py --steps 3 --warmup 2 --no-ckpt > gpurun_out/prof_head.log 2>&1 || exit $?
