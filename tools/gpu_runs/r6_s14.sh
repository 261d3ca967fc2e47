#!/bin/bash
# Round 6 session 14: host enqueue vs GPU time of the eager step with every data-parallel collective issued over
# RCCL at world 1 (force_comm), ResNet-50 and Inception-v3, fp32 and bf16 wire; the no-comm baseline.
set -o pipefail
mkdir -p gpurun_out/r6
for m in resnet_v1_50 inception_v3_slim_old; do
  timeout -k 10 200 python -u tools/cpu_overhead.py --model $m --steps 20 >> gpurun_out/r6/r6_s14_cpu_overhead.log 2>&1 || { tail -20 gpurun_out/r6/r6_s14_cpu_overhead.log; exit 1; }
  timeout -k 10 200 python -u tools/cpu_overhead.py --model $m --steps 20 --force-comm >> gpurun_out/r6/r6_s14_cpu_overhead.log 2>&1 || { tail -20 gpurun_out/r6/r6_s14_cpu_overhead.log; exit 1; }
  timeout -k 10 200 python -u tools/cpu_overhead.py --model $m --steps 20 --force-comm --grad-comm bf16 >> gpurun_out/r6/r6_s14_cpu_overhead.log 2>&1 || { tail -20 gpurun_out/r6/r6_s14_cpu_overhead.log; exit 1; }
done
grep -v "amdgpu.ids\|NCCL\|^\[" gpurun_out/r6/r6_s14_cpu_overhead.log
