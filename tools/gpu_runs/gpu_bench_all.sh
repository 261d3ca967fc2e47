#!/bin/bash
# Every BASELINE config on one MI355X (bench.py, K=20 W=5); one value line per model.
set -o pipefail
mkdir -p gpurun_out
for m in resnet_v1_50 inception_v3_slim_old vgg_16 lenet; do
  timeout -k 10 300 python bench.py --model $m --steps 20 --warmup 5 > gpurun_out/all_$m.log 2>&1 || { echo "bench $m failed"; tail -20 gpurun_out/all_$m.log; exit 1; }
  echo "$m $(grep -o '"value": [0-9.]*, "unit": "images/sec", "n_gpus": [0-9]*, "steps": [0-9]*, "warmup": [0-9]*, "ms_per_step": [0-9.]*' gpurun_out/all_$m.log)"
done
