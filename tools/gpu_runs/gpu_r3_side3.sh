#!/bin/bash
# Direct 3x3 kernel with LDS-DMA dgrad post-op inputs: numerics, Inception A/B, bench, timeline.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_fused_ops_gpu.py -k "direct3x3 or chain or full_window" > gpurun_out/side3_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/side3_tests.log; exit 1; }
tail -1 gpurun_out/side3_tests.log
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_fused_gpu.py tests/test_zoo_gpu.py > gpurun_out/side3_suites.log 2>&1 || { echo "suites failed"; tail -40 gpurun_out/side3_suites.log; exit 1; }
tail -1 gpurun_out/side3_suites.log
MODEL=inception_v3_slim_old VARIANTS="direct=dir3:1;gemm=dir3:0" ROUNDS=6 timeout -k 10 400 python -u tools/ab_step.py > gpurun_out/dir3_inc3.log 2>&1 || { tail -30 gpurun_out/dir3_inc3.log; exit 1; }
tail -3 gpurun_out/dir3_inc3.log
bash tools/gpu_runs/gpu_r3_inc.sh
