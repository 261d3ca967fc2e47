#!/bin/bash
# Round 6 session 1: baseline on this round's box - default bench, and a kernel trace of the captured ResNet-50
# step with the conv tile log (shape -> kernel map for the per-layer conv times).
set -o pipefail
mkdir -p gpurun_out/r6
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 200 python -u bench.py > gpurun_out/r6/r6_s1_bench_default.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/r6/r6_s1_bench_default.log; exit 1; }
tail -1 gpurun_out/r6/r6_s1_bench_default.log | cut -c1-200
rm -rf gpurun_out/r6/prof_s1
cd /tmp && DTM_TILE_LOG=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r6/prof_s1 -o run --output-format csv -- python3 $R/bench.py --steps 4 --warmup 2 > $R/gpurun_out/r6/r6_s1_prof.log 2>&1 || { echo "prof failed"; tail -5 $R/gpurun_out/r6/r6_s1_prof.log; exit 1; }
cd $R
f=$(find gpurun_out/r6/prof_s1 -name "*kernel_stats.csv" | head -1); cp "$f" gpurun_out/r6/r6_s1_resnet50_kernel_stats.csv
t=$(find gpurun_out/r6/prof_s1 -name "*kernel_trace.csv" | head -1); python3 tools/step_timeline.py "$t" > gpurun_out/r6/r6_s1_timeline_resnet.txt; tail -1 gpurun_out/r6/r6_s1_timeline_resnet.txt
rm -rf gpurun_out/r6/prof_s1
echo done
