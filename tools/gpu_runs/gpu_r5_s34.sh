#!/bin/bash
# Round 5 session 34: Inception-v3 captured-step kernel trace -> per-launch timeline (reduce-class launch census).
set -o pipefail
mkdir -p gpurun_out/r5
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
rm -rf gpurun_out/r5/prof_s34
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r5/prof_s34 -o run --output-format csv -- python3 $R/bench.py --model inception_v3_slim_old --steps 4 --warmup 3 > $R/gpurun_out/r5/prof_s34.log 2>&1 || { echo "prof failed"; tail -20 $R/gpurun_out/r5/prof_s34.log; exit 1; }
cd $R
f=$(find gpurun_out/r5/prof_s34 -name "*kernel_stats.csv" | head -1); cp "$f" gpurun_out/r5/r5_s34_inception_kernel_stats.csv
t=$(find gpurun_out/r5/prof_s34 -name "*kernel_trace.csv" | head -1); python3 tools/step_timeline.py "$t" > gpurun_out/r5/r5_s34_timeline_inception.txt; tail -1 gpurun_out/r5/r5_s34_timeline_inception.txt
rm -rf gpurun_out/r5/prof_s34
echo done
