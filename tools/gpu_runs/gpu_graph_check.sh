#!/bin/bash
# hipGraph step: numerics vs eager, multi-rank BSP on HIP kernels, then eager-vs-graph bench per model.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_engine.py tests/test_distributed.py -m gpu > gpurun_out/graph_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/graph_tests.log; exit 1; }
tail -8 gpurun_out/graph_tests.log
for m in lenet vgg_16 resnet_v1_50; do
  for g in 0 1; do
    timeout -k 10 300 python bench.py --model $m --steps ${STEPS:-20} --warmup 5 --graph $g > gpurun_out/bench_${m}_g$g.log 2>&1 || { echo "bench $m g$g failed"; tail -30 gpurun_out/bench_${m}_g$g.log; exit 1; }
    echo "$m graph=$g: $(grep -o '"value": [0-9.]*, "unit": "[^"]*", "n_gpus": [0-9]*, "steps": [0-9]*, "warmup": [0-9]*, "ms_per_step": [0-9.]*' gpurun_out/bench_${m}_g$g.log)"
  done
done
