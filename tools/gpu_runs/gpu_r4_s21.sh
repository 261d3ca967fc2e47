#!/bin/bash
# Round 4 closing run: smoke, ResNet-50 bench, Inception-v3 kernel trace (stats + one-step timeline) on the final code.
set -o pipefail
mkdir -p gpurun_out/r4
export TMPDIR=/tmp
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4/r4_close_smoke.log 2>&1 || { tail -20 gpurun_out/r4/r4_close_smoke.log; exit 1; }
tail -1 gpurun_out/r4/r4_close_smoke.log
timeout -k 10 200 python -u bench.py --steps 30 --warmup 5 > gpurun_out/r4/r4_close_bench_resnet.log 2>&1 || { tail -20 gpurun_out/r4/r4_close_bench_resnet.log; exit 1; }
tail -1 gpurun_out/r4/r4_close_bench_resnet.log | cut -c1-200
rm -rf gpurun_out/r4/prof_inc
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r4/prof_inc -o run -- python3 $GRAFT_REPO_ROOT/bench.py --model inception_v3_slim_old --steps 5 --warmup 3 > $GRAFT_REPO_ROOT/gpurun_out/r4/r4_close_prof_inception.log 2>&1 || { echo "prof failed"; tail -30 $GRAFT_REPO_ROOT/gpurun_out/r4/r4_close_prof_inception.log; exit 1; }
cd $GRAFT_REPO_ROOT
f=$(find gpurun_out/r4/prof_inc -name "*kernel_trace.csv" | head -1)
python3 tools/step_timeline.py "$f" > gpurun_out/r4/r4_close_timeline_inception.txt
tail -1 gpurun_out/r4/r4_close_timeline_inception.txt
s=$(find gpurun_out/r4/prof_inc -name "*kernel_stats.csv" | head -1)
cp "$s" gpurun_out/r4/r4_close_inception_kernel_stats.csv
rm -rf gpurun_out/r4/prof_inc
