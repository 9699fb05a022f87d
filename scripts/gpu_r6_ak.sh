#!/bin/bash
# Round 6, session AK: no-GQA dK RoPE backward per 16-B chunk in the dK/dV row stores: flash tests,
# GPT-2 graph benches A/B (FT_FLASH_DIRECT_ROPE).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_flash_attn_gpu.py > gpurun_out/r6ak_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r6ak_tests.log; [ $rc -eq 0 ] || exit $rc
for m in gpt2-small gpt2-medium; do
  for v in 1 0 1 0; do
    FT_FLASH_DIRECT_ROPE=$v timeout -k 10 300 python -u bench.py --model $m --vocab-size 50304 --graph --steps 50 --warmup 5 --no-ckpt > gpurun_out/r6ak_b.json 2>gpurun_out/r6ak_b.err || { tail -3 gpurun_out/r6ak_b.err; exit 1; }
    echo "$m direct_rope=$v $(python3 -c "import json;d=json.loads(open('gpurun_out/r6ak_b.json').read().strip().splitlines()[-1]);print(d['ms_per_step'], d.get('sclk_mhz_p50'))")" >> gpurun_out/r6ak_bench.log
  done
done
cat gpurun_out/r6ak_bench.log
