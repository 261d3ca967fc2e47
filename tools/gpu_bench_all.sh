#!/bin/bash
# Every BASELINE config on one MI355X (bench.py, K=20 W=5) + a ResNet-50 kernel-stat profile.
set -o pipefail
mkdir -p gpurun_out
for m in resnet_v1_50 inception_v3_slim_old vgg_16 lenet; do
  timeout -k 10 300 python bench.py --model $m --steps ${STEPS:-20} --warmup 5 > gpurun_out/all_$m.log 2>&1 || { echo "bench $m failed"; tail -20 gpurun_out/all_$m.log; exit 1; }
  grep '"value"' gpurun_out/all_$m.log
done
bash tools/gpu_session.sh prof > gpurun_out/all_prof.log 2>&1 || { tail -20 gpurun_out/all_prof.log; exit 1; }
python3 tools/prof_summary.py $(find gpurun_out/prof -name "*kernel_stats.csv" | head -1) 5 30
