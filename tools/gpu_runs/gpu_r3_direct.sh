#!/bin/bash
# Direct 3x3 conv kernel: numerics first (its own tests, then the conv suites), then step A/B and benches.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_fused_ops_gpu.py -k "direct3x3 or full_window" > gpurun_out/direct_tests.log 2>&1 || { echo "direct tests failed"; tail -40 gpurun_out/direct_tests.log; exit 1; }
tail -1 gpurun_out/direct_tests.log
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_fused_ops_gpu.py tests/test_fused_gpu.py tests/test_zoo_gpu.py > gpurun_out/direct_suites.log 2>&1 || { echo "suites failed"; tail -40 gpurun_out/direct_suites.log; exit 1; }
tail -1 gpurun_out/direct_suites.log
true
true
MODEL=inception_v3_slim_old VARIANTS="direct=dir3:1;gemm=dir3:0" ROUNDS=4 timeout -k 10 400 python -u tools/ab_step.py > gpurun_out/dir3_inc.log 2>&1 || { tail -30 gpurun_out/dir3_inc.log; exit 1; }
tail -3 gpurun_out/dir3_inc.log
timeout -k 10 300 python bench.py --model inception_v3_slim_old > gpurun_out/bench_inc.log 2>&1 || { tail -20 gpurun_out/bench_inc.log; exit 1; }
grep '"value"' gpurun_out/bench_inc.log | cut -c1-200
timeout -k 10 300 python bench.py > gpurun_out/bench_rn.log 2>&1 || { tail -20 gpurun_out/bench_rn.log; exit 1; }
grep '"value"' gpurun_out/bench_rn.log | cut -c1-200
VARIANTS="w0=wwide:0;w3=wwide:3" ROUNDS=5 timeout -k 10 400 python -u tools/ab_step.py > gpurun_out/wwide3_rn.log 2>&1 || { tail -30 gpurun_out/wwide3_rn.log; exit 1; }
tail -3 gpurun_out/wwide3_rn.log
