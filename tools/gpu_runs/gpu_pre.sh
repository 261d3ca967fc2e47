#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_fused_gpu.py tests/test_fused_ops_gpu.py tests/test_dgrad_decomposition.py -m gpu > gpurun_out/t_pre.log 2>&1 || { tail -40 gpurun_out/t_pre.log; exit 1; }
tail -2 gpurun_out/t_pre.log
VARIANTS="pre=;nopre=pre:0" timeout -k 10 300 python -u tools/ab_step.py > gpurun_out/r2_ab_pre_side.log 2>&1 || { tail -20 gpurun_out/r2_ab_pre_side.log; exit 1; }
tail -2 gpurun_out/r2_ab_pre_side.log
MODEL=inception_v3_slim_old STEPS=15 ROUNDS=4 VARIANTS="pre=;nopre=pre:0" timeout -k 10 300 python -u tools/ab_step.py > gpurun_out/r2_ab_pre_side_inception.log 2>&1 || { tail -20 gpurun_out/r2_ab_pre_side_inception.log; exit 1; }
tail -2 gpurun_out/r2_ab_pre_side_inception.log
