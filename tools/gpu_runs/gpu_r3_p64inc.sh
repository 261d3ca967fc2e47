#!/bin/bash
# Eager A/B of the pipelined 64x128 wgrad tile on Inception-v3; ResNet-50 bench; Inception-v3 bench (one captured
# graph per process, the product path) last.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
MODEL=inception_v3_slim_old VARIANTS="base=;p1=wp64:1;p2=wp64:2" ROUNDS=6 timeout -k 10 500 python -u tools/ab_step.py > gpurun_out/r3_ab_wgrad_p64_inception.log 2>&1 || { tail -30 gpurun_out/r3_ab_wgrad_p64_inception.log; exit 1; }
tail -3 gpurun_out/r3_ab_wgrad_p64_inception.log
timeout -k 10 300 python bench.py > gpurun_out/r3_bench_resnet.log 2>&1 || { tail -20 gpurun_out/r3_bench_resnet.log; exit 1; }
tail -1 gpurun_out/r3_bench_resnet.log
timeout -k 10 300 python bench.py --model inception_v3_slim_old > gpurun_out/r3_bench_inception.log 2>&1 || { tail -20 gpurun_out/r3_bench_inception.log; exit 1; }
tail -1 gpurun_out/r3_bench_inception.log
