#!/bin/bash
# Kernel-stat profiles of the non-headline BASELINE configs (Inception-v3 old slim, VGG-16 CIFAR geometry).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for m in ${MODELS:-inception_v3_slim_old vgg_16}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$m -o run --output-format csv -- python3 $R/bench.py --model $m --steps 3 --warmup 2 > $R/gpurun_out/prof_$m.log 2>&1 || { echo "prof $m failed"; tail -20 $R/gpurun_out/prof_$m.log; exit 1; }
  f=$(find $R/gpurun_out/prof_$m -name "*kernel_stats.csv" | head -1)
  echo "== $m"; grep '"value"' $R/gpurun_out/prof_$m.log | cut -c1-200
  python3 $R/tools/prof_summary.py $f 5 30
done
