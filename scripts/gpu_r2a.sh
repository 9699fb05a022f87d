#!/bin/bash
# Re-verify the rebuilt tree on MI355X: GPU tests, smoke, bench, per-GEMM timings
export TMPDIR=/tmp
mkdir -p gpurun_out
S=scripts/gpu_check.sh
$S gputests 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread || exit 1
$S smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
$S bench 600 python bench.py || exit 1
$S gemm_shapes 300 python scripts/gemm_shapes_bench.py || exit 1
export PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_VERBOSE=1
PYTORCH_TUNABLEOP_FILENAME=gpurun_out/tunable_gemm%d.csv $S gemm_shapes_tuned 600 python scripts/gemm_shapes_bench.py || exit 1
PYTORCH_TUNABLEOP_FILENAME=gpurun_out/tunable_bench%d.csv $S bench_tuned 900 python bench.py --warmup 3 --steps 10 || exit 1
