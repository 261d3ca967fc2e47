#!/bin/bash
# Round 6 session 8: serial (no side stream) ResNet-50 step kernel trace + tile log: each kernel's isolated time, for
# the per-category work accounting; and the same-process A/B of the side stream itself.
set -o pipefail
mkdir -p gpurun_out/r6
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
rm -rf gpurun_out/r6/prof_s8
cd /tmp && DTM_TILE_LOG=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r6/prof_s8 -o run --output-format csv -- python3 $R/bench.py --steps 4 --warmup 2 --wgrad-stream 0 > $R/gpurun_out/r6/r6_s8_prof.log 2>&1 || { echo "prof failed"; tail -5 $R/gpurun_out/r6/r6_s8_prof.log; exit 1; }
cd $R
t=$(find gpurun_out/r6/prof_s8 -name "*kernel_trace.csv" | head -1); python3 tools/step_timeline.py "$t" > gpurun_out/r6/r6_s8_timeline_serial.txt; tail -1 gpurun_out/r6/r6_s8_timeline_serial.txt
rm -rf gpurun_out/r6/prof_s8
VARIANTS="side=;serial=wgs:0" ROUNDS=4 timeout -k 10 300 python -u tools/ab_step.py > gpurun_out/r6/r6_s8_ab_side.log 2>&1 || { tail -20 gpurun_out/r6/r6_s8_ab_side.log; exit 1; }
tail -2 gpurun_out/r6/r6_s8_ab_side.log
