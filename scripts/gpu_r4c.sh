#!/bin/bash
# RCCL code path of bench.py at full 8B scale on a 1-rank process group (zero1 / allreduce),
# then a fresh kernel-trace profile of HEAD
export TMPDIR=/tmp
mkdir -p gpurun_out
S=scripts/gpu_check.sh
FT_FORCE_DIST=1 $S rc_zero1 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29611 bench.py --dp-mode zero1 || exit 1
FT_FORCE_DIST=1 $S rc_allreduce 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29612 bench.py --dp-mode allreduce || exit 1
rm -rf gpurun_out/kprof4
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/kprof4 -o run --output-format csv -- python3 bench.py --steps 4 --warmup 2 > gpurun_out/kprof4.log 2>&1 || exit 1
echo "prof rc=0"; tail -2 gpurun_out/kprof4.log
