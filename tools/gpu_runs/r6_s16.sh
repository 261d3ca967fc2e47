#!/bin/bash
# Round 6 session 16: host enqueue vs GPU time with every collective issued over RCCL (world 1): eager vs the step
# captured with its collectives (graph_comm), ResNet-50 and Inception-v3.
set -o pipefail
mkdir -p gpurun_out/r6
L=gpurun_out/r6/r6_s16_cpu_overhead_comm.log
for m in resnet_v1_50 inception_v3_slim_old; do
  timeout -k 10 200 python -u tools/cpu_overhead.py --model $m --steps 20 --force-comm >> $L 2>&1 || { tail -20 $L; exit 1; }
  timeout -k 10 200 python -u tools/cpu_overhead.py --model $m --steps 20 --force-comm --graph >> $L 2>&1 || { tail -20 $L; exit 1; }
  timeout -k 10 200 python -u tools/cpu_overhead.py --model $m --steps 20 --force-comm --graph --grad-comm bf16 >> $L 2>&1 || { tail -20 $L; exit 1; }
done
grep "host enqueue" $L
