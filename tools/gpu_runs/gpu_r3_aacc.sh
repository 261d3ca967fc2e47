#!/bin/bash
# Per-worker activation-backward sums in the persistent kernels: numerics, A/B (both models), timelines.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_fused_ops_gpu.py tests/test_kernels_gpu.py tests/test_fused_gpu.py tests/test_zoo_gpu.py tests/test_trajectory_gpu.py > gpurun_out/aacc_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/aacc_tests.log; exit 1; }
tail -1 gpurun_out/aacc_tests.log
MODEL=inception_v3_slim_old VARIANTS="direct=dir3:1;gemm=dir3:0" ROUNDS=6 timeout -k 10 400 python -u tools/ab_step.py > gpurun_out/dir3_inc4.log 2>&1 || { tail -30 gpurun_out/dir3_inc4.log; exit 1; }
tail -3 gpurun_out/dir3_inc4.log
VARIANTS="base=;sact0=sact:0" ROUNDS=5 timeout -k 10 400 python -u tools/ab_step.py > gpurun_out/sact_rn.log 2>&1 || { tail -30 gpurun_out/sact_rn.log; exit 1; }
tail -3 gpurun_out/sact_rn.log
bash tools/gpu_runs/gpu_r3_inc.sh
grep "conv3x3_direct" gpurun_out/r3_timeline_inc.txt | cut -c1-110
