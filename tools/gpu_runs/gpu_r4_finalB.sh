#!/bin/bash
# Round-4 final evidence B: smoke, then every BASELINE config's bench.
set -o pipefail
mkdir -p gpurun_out/r4
export TMPDIR=/tmp
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4/r4_final_smoke.log 2>&1 || { tail -20 gpurun_out/r4/r4_final_smoke.log; exit 1; }
tail -1 gpurun_out/r4/r4_final_smoke.log
for m in resnet_v1_50 inception_v3_slim_old vgg_16 lenet; do
  timeout -k 10 300 python bench.py --model $m > gpurun_out/r4/r4_final_bench_$m.log 2>&1 || { tail -20 gpurun_out/r4/r4_final_bench_$m.log; exit 1; }
  tail -1 gpurun_out/r4/r4_final_bench_$m.log | cut -c1-220
done
