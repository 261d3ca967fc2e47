#!/bin/bash
# full-window dgrad GEMM + stem-only wide wgrad: numerics, A/B, benches.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_fused_ops_gpu.py tests/test_zoo_gpu.py > gpurun_out/misc_tests.log 2>&1 || { tail -30 gpurun_out/misc_tests.log; exit 1; }
tail -1 gpurun_out/misc_tests.log
VARIANTS="stem=wwide:2;narrow=wwide:0" ROUNDS=5 timeout -k 10 400 python -u tools/ab_step.py > gpurun_out/wwide2_rn.log 2>&1 || { tail -30 gpurun_out/wwide2_rn.log; exit 1; }
tail -3 gpurun_out/wwide2_rn.log
timeout -k 10 300 python bench.py --model inception_v3_slim_old > gpurun_out/bench_inc.log 2>&1 || { tail -20 gpurun_out/bench_inc.log; exit 1; }
grep '"value"' gpurun_out/bench_inc.log | cut -c1-200
timeout -k 10 300 python bench.py > gpurun_out/bench_rn.log 2>&1 || { tail -20 gpurun_out/bench_rn.log; exit 1; }
grep '"value"' gpurun_out/bench_rn.log | cut -c1-200
