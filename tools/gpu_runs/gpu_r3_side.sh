#!/bin/bash
# Side-stream weight gradients: full GPU tests, knob interactions, bench (ResNet-50, Inception eager vs graph).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > gpurun_out/side_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 gpurun_out/side_tests.log; exit 1; }
tail -1 gpurun_out/side_tests.log
VARIANTS="base=;b1x1off=b1x1:0;bnoutoff=bnout:0;wocc3=wtile:-1:3;nowgs=wgs:0" ROUNDS=4 timeout -k 10 400 python -u tools/ab_step.py > gpurun_out/side_step.log 2>&1 || { tail -30 gpurun_out/side_step.log; exit 1; }
tail -5 gpurun_out/side_step.log
timeout -k 10 300 python bench.py > gpurun_out/bench_rn.log 2>&1 || { tail -20 gpurun_out/bench_rn.log; exit 1; }
grep '"value"' gpurun_out/bench_rn.log | cut -c1-200
timeout -k 10 300 python bench.py --model inception_v3_slim_old > gpurun_out/bench_inc.log 2>&1 || { tail -20 gpurun_out/bench_inc.log; exit 1; }
grep '"value"' gpurun_out/bench_inc.log | cut -c1-200
timeout -k 10 300 python bench.py --model inception_v3_slim_old --graph 0 > gpurun_out/bench_inc_eager.log 2>&1 || { tail -20 gpurun_out/bench_inc_eager.log; exit 1; }
grep '"value"' gpurun_out/bench_inc_eager.log | cut -c1-200
