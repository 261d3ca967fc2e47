#!/bin/bash
# Per-kernel profile of the ResNet-50 step with the stem stream on / off.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in 1 0; do
VARIANTS="s=sstr:$v" ROUNDS=1 STEPS=3 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_stem$v -o run -- python3 -u tools/ab_step.py > gpurun_out/stem_prof$v.log 2>&1 || { tail -30 gpurun_out/stem_prof$v.log; exit 1; }
f=$(ls gpurun_out/prof_stem$v/run_kernel_stats.csv gpurun_out/prof_stem$v/*/run_kernel_stats.csv 2>/dev/null | head -1)
echo "== sstr=$v $f"; python3 tools/prof_summary.py "$f" 5 14 | grep -i "total\|stream\|pipe\|stem"
done
