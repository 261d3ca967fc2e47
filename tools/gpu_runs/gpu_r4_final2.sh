#!/bin/bash
# Round-4 final evidence part 2: 8-rank gloo rehearsal of the driver's launch, ResNet-50 kernel trace.
set -o pipefail
mkdir -p gpurun_out/r4
export TMPDIR=/tmp
timeout -k 10 600 python bench.py --gpus 8 --dist-backend gloo --batch 32 --steps 3 --warmup 2 > gpurun_out/r4/r4_final_gloo8.log 2>&1 || { tail -30 gpurun_out/r4/r4_final_gloo8.log; exit 1; }
tail -1 gpurun_out/r4/r4_final_gloo8.log | cut -c1-300
rm -rf gpurun_out/r4/prof_final
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r4/prof_final -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 3 > $GRAFT_REPO_ROOT/gpurun_out/r4/r4_final_prof.log 2>&1 || { echo "prof failed"; tail -30 $GRAFT_REPO_ROOT/gpurun_out/r4/r4_final_prof.log; exit 1; }
cd $GRAFT_REPO_ROOT
f=$(find gpurun_out/r4/prof_final -name "*kernel_trace.csv" | head -1)
python3 tools/step_timeline.py "$f" > gpurun_out/r4/r4_final_timeline_resnet.txt
tail -1 gpurun_out/r4/r4_final_timeline_resnet.txt
s=$(find gpurun_out/r4/prof_final -name "*kernel_stats.csv" | head -1)
cp "$s" gpurun_out/r4/r4_final_resnet50_kernel_stats.csv
rm -rf gpurun_out/r4/prof_final
