#!/bin/bash
# Round 5 session 11: Inception-v3 captured-step kernel trace -> per-launch timeline (reduce-class launch census).
set -o pipefail
mkdir -p gpurun_out/r5
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
rm -rf gpurun_out/r5/prof_s11
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r5/prof_s11 -o run --output-format csv -- python3 $R/bench.py --model inception_v3_slim_old --steps 4 --warmup 3 > $R/gpurun_out/r5/prof_s11.log 2>&1 || { echo "prof failed"; tail -20 $R/gpurun_out/r5/prof_s11.log; exit 1; }
cd $R
f=$(find gpurun_out/r5/prof_s11 -name "*kernel_stats.csv" | head -1); cp "$f" gpurun_out/r5/r5_inception_kernel_stats.csv
t=$(find gpurun_out/r5/prof_s11 -name "*kernel_trace.csv" | head -1); python3 tools/step_timeline.py "$t" > gpurun_out/r5/r5_timeline_inception.txt; tail -1 gpurun_out/r5/r5_timeline_inception.txt
rm -rf gpurun_out/r5/prof_s11
echo done
