#!/bin/bash
# Round 6, session AC: the 3-kernel GQA flash backward (dK/dV first with its own delta, dQ + fold):
# flash tests (bitwise against the 4-kernel order), the backward A/B at the 8B layer, a kernel trace.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_flash_attn_gpu.py > gpurun_out/r6ac_tests.log 2>&1
rc=$?; tail -4 gpurun_out/r6ac_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/flash_fold3_ab.py > gpurun_out/r6ac_fold3_ab.log 2>&1 || { tail -5 gpurun_out/r6ac_fold3_ab.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r6ac_fold3_ab.log
