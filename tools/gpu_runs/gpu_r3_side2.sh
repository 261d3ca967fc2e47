#!/bin/bash
# Side-stream weight gradients inside the hipGraph-captured step (Inception-v3, VGG-16).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for m in inception_v3_slim_old vgg_16; do
timeout -k 10 300 python bench.py --model $m > gpurun_out/bench_g0_$m.log 2>&1 || { tail -20 gpurun_out/bench_g0_$m.log; exit 1; }
grep '"value"' gpurun_out/bench_g0_$m.log | cut -c1-180
DTM_WGRAD_STREAM_GRAPH=1 timeout -k 10 300 python bench.py --model $m > gpurun_out/bench_g1_$m.log 2>&1 || { tail -20 gpurun_out/bench_g1_$m.log; exit 1; }
grep '"value"' gpurun_out/bench_g1_$m.log | cut -c1-180
done
