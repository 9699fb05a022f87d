#!/bin/bash
# RCCL data-parallel path on one GPU: the 1-rank process-group test, then the 8B bench locally
# and through a 1-rank RCCL group (ZeRO-1 / all-reduce): the collectives' local overhead.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/dp1
C="bash scripts/gpu_check.sh"
# $C dp1/test 300 python -u -m pytest tests/test_dp_rccl_gpu.py -x -v --timeout 250 --timeout-method thread || exit $?
# grep -q "passed" gpurun_out/dp1/test.log && ! grep -q "failed" gpurun_out/dp1/test.log || exit 1
$C dp1/local 300 python bench.py --no-ckpt --steps 10 --warmup 3 || exit $?
export FT_FORCE_DIST=1
TR="python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29517"
$C dp1/zero1 300 $TR bench.py --no-ckpt --steps 10 --warmup 3 --dp-mode zero1 || exit $?
$C dp1/allreduce 300 $TR bench.py --no-ckpt --steps 10 --warmup 3 --dp-mode allreduce || exit $?
