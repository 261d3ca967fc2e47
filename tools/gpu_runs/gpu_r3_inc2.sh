#!/bin/bash
# Inception: direct 3x3 only without dgrad post-ops; A/B + bench + timeline.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
MODEL=inception_v3_slim_old VARIANTS="direct=dir3:1;gemm=dir3:0" ROUNDS=6 timeout -k 10 400 python -u tools/ab_step.py > gpurun_out/dir3_inc2.log 2>&1 || { tail -30 gpurun_out/dir3_inc2.log; exit 1; }
tail -3 gpurun_out/dir3_inc2.log
timeout -k 10 300 python bench.py --model inception_v3_slim_old > gpurun_out/bench_inc.log 2>&1 || { tail -20 gpurun_out/bench_inc.log; exit 1; }
grep '"value"' gpurun_out/bench_inc.log | cut -c1-200
bash tools/gpu_runs/gpu_r3_inc.sh
