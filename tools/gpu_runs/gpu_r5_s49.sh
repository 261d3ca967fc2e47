#!/bin/bash
# Round 5 session 49: host enqueue time vs GPU time of the eager ResNet-50 / Inception-v3 steps (tools/cpu_overhead.py).
set -o pipefail
mkdir -p gpurun_out/r5
timeout -k 10 200 python -u tools/cpu_overhead.py --model resnet_v1_50 > gpurun_out/r5/r5_s49_cpu_overhead.log 2>&1 || { tail -5 gpurun_out/r5/r5_s49_cpu_overhead.log; exit 1; }
timeout -k 10 200 python -u tools/cpu_overhead.py --model inception_v3_slim_old >> gpurun_out/r5/r5_s49_cpu_overhead.log 2>&1 || { tail -5 gpurun_out/r5/r5_s49_cpu_overhead.log; exit 1; }
grep "host enqueue" gpurun_out/r5/r5_s49_cpu_overhead.log
echo done
