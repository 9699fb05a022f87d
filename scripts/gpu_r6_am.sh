#!/bin/bash
# Round 6, session AM: dQ RoPE backward with float2 table loads: flash tests, flash backward timing
# (8B layer with RoPE), GPT-2 graph benches.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_flash_attn_gpu.py tests/test_w4_paths_gpu.py > gpurun_out/r6am_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r6am_tests.log; [ $rc -eq 0 ] || exit $rc
FOLD3_ONLY=0 timeout -k 10 300 python -u scripts/flash_fold3_ab.py 2>&1 | grep -v amdgpu.ids
for m in gpt2-small gpt2-medium; do
  for r in 1 2; do
    timeout -k 10 300 python -u bench.py --model $m --vocab-size 50304 --graph --steps 50 --warmup 5 --no-ckpt > gpurun_out/r6am_b.json 2>gpurun_out/r6am_b.err || { tail -3 gpurun_out/r6am_b.err; exit 1; }
    echo "$m $(python3 -c "import json;d=json.loads(open('gpurun_out/r6am_b.json').read().strip().splitlines()[-1]);print(d['ms_per_step'], d.get('sclk_mhz_p50'))")"
  done
done
