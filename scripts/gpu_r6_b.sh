#!/bin/bash
# Round 6, session B: bisect the ZeRO-1 capture segfault (capture_collectives_probe.py).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
P=scripts/capture_collectives_probe.py
timeout -k 10 200 python -u $P --only side_roundtrip,side_roundtrip_rs_first > gpurun_out/r6b_capture_probe.log 2>&1
grep -E "^=== " gpurun_out/r6b_capture_probe.log
