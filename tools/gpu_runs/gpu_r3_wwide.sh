#!/bin/bash
# 64x256 register-staged wgrad tile only for the BN-fused (stem) wgrad: step A/B + stem wgrad kernel time.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
VARIANTS="stem=wwide:2;narrow=wwide:0" ROUNDS=5 timeout -k 10 400 python -u tools/ab_step.py > gpurun_out/wwide2_rn.log 2>&1 || { tail -30 gpurun_out/wwide2_rn.log; exit 1; }
tail -3 gpurun_out/wwide2_rn.log
for v in 2 0; do
VARIANTS="s=wwide:$v" ROUNDS=1 STEPS=3 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_ww$v -o run -- python3 -u tools/ab_step.py > gpurun_out/ww_prof$v.log 2>&1 || { tail -30 gpurun_out/ww_prof$v.log; exit 1; }
f=$(ls gpurun_out/prof_ww$v/run_kernel_stats.csv gpurun_out/prof_ww$v/*/run_kernel_stats.csv 2>/dev/null | head -1)
echo "== wwide=$v"; python3 tools/prof_summary.py "$f" 5 60 | grep -i "total\|conv_wgrad_kernel"
done
