#!/bin/bash
# Round-4 probe: LDS wait-state counters of the w4 layouts, per-knob step A/B, kernel stats of the step
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU --kernel-trace --output-format csv -d gpurun_out/pmc_w4t2 -o w4t -- python3 scripts/w4t_pmc_probe.py > gpurun_out/r4_w4t_pmc2_run.log 2>&1 || exit $?
python3 scripts/pmc_summary.py gpurun_out/pmc_w4t2 > gpurun_out/r4_w4t_pmc2.txt
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r4 -o run --output-format csv -- python3 bench.py --steps 5 --warmup 3 --no-ckpt > gpurun_out/r4_prof.log 2>&1 || exit $?
python3 scripts/prof_timeline.py gpurun_out/prof_r4/run_kernel_trace.csv --steps 3 > gpurun_out/r4_prof_timeline.txt
timeout -k 10 600 python -u scripts/ab_step.py --knobs w4bwd,psums,w4head --rounds 2 --steps 6 > gpurun_out/r4_ab_parts.log 2>&1
