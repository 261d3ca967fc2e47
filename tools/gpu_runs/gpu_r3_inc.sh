#!/bin/bash
# Inception-v3 step profile (bench config: hipGraph, batch 128): kernel stats + step timeline.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/prof_inc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_inc -o run -- python3 bench.py --model inception_v3_slim_old --steps 3 --warmup 3 > gpurun_out/prof_inc.log 2>&1 || { echo "prof failed"; tail -30 gpurun_out/prof_inc.log; exit 1; }
f=$(find gpurun_out/prof_inc -name "*kernel_trace.csv" | head -1)
python3 tools/step_timeline.py "$f" > gpurun_out/r3_timeline_inc.txt
tail -1 gpurun_out/r3_timeline_inc.txt
