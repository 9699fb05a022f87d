#!/bin/bash
# round-end rehearsal on HEAD: full GPU suite, smoke, default bench, bench + checkpoint save
export TMPDIR=/tmp
mkdir -p gpurun_out
S=scripts/gpu_check.sh
$S fa_test 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread || exit 1
$S fa_smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
$S fa_bench 300 python bench.py || exit 1
$S fa_bench_ck 400 python bench.py --ckpt-dir /tmp/ftck --steps 5 || exit 1
