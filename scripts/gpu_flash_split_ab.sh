#!/bin/bash
# Flash key-split A/B: kernel timings at the GPT-2 / 8B layer shapes, then whole steps
# (GPT-2-small/-medium with the HIP graph, Llama-3-8B) with the splits on (default) and off.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/fsplit
C="bash scripts/gpu_check.sh"
$C fsplit/kern 200 bash -c 'for a in "2048 12 12 64" "2048 16 16 64" "2048 32 8 128" "16384 4 1 128"; do python scripts/flash_bench.py $a || exit 1; done' || exit $?
for m in gpt2-small gpt2-medium; do
  $C fsplit/${m}_on 200 python bench.py --model $m --graph --no-ckpt --steps 30 --warmup 5 || exit $?
  FT_FLASH_FWD_SPLIT=0 FT_FLASH_DQ_SPLIT=0 FT_FLASH_KV_SPLIT=0 $C fsplit/${m}_off 200 python bench.py --model $m --graph --no-ckpt --steps 30 --warmup 5 || exit $?
done
$C fsplit/8b_on 300 python bench.py --no-ckpt --steps 10 --warmup 3 || exit $?
FT_FLASH_DQ_SPLIT=0 $C fsplit/8b_off 300 python bench.py --no-ckpt --steps 10 --warmup 3 || exit $?
$C fsplit/8b_on2 300 python bench.py --no-ckpt --steps 10 --warmup 3 || exit $?
