#!/bin/bash
# Round 5 session 46: ResNet-50 captured step with kernel + memory-copy traces (what fills the idle gaps on the main
# stream at the start of the backward: 39.6 / 21.0 us in r5_s45_timeline_resnet.txt).
set -o pipefail
mkdir -p gpurun_out/r5
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $R/gpurun_out/r5/prof_s46 -o run --output-format csv -- python3 $R/bench.py --steps 4 --warmup 3 > $R/gpurun_out/r5/prof_s46.log 2>&1 || { echo "prof failed"; exit 1; }
cd $R
find gpurun_out/r5/prof_s46 -name "*.csv" | head
t=$(find gpurun_out/r5/prof_s46 -name "*kernel_trace.csv" | head -1); cp "$t" gpurun_out/r5/r5_s46_kernel_trace.csv
m=$(find gpurun_out/r5/prof_s46 -name "*memory_copy_trace.csv" | head -1); [ -n "$m" ] && cp "$m" gpurun_out/r5/r5_s46_memcpy_trace.csv
rm -rf gpurun_out/r5/prof_s46
ls -la gpurun_out/r5/r5_s46_*
echo done
