#!/bin/bash
# kernel statistics of the captured Inception-v3 bench step (after the round-6 stem kernels)
set -o pipefail
mkdir -p gpurun_out/r6
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r6/prof39 -o run -- python3 $R/bench.py --model inception_v3_slim_old --steps 10 --warmup 3 > $R/gpurun_out/r6/r6_s39_prof_bench.log 2>&1 || { echo "profile failed"; tail -5 $R/gpurun_out/r6/r6_s39_prof_bench.log; exit 1; }
cd $R
f=$(find gpurun_out/r6/prof39 -name "*kernel_stats.csv" | head -1); cp "$f" gpurun_out/r6/r6_s39_inception_kernel_stats.csv
find gpurun_out/r6/prof39 -name "*.csv" -delete
head -30 gpurun_out/r6/r6_s39_inception_kernel_stats.csv | cut -c1-150
