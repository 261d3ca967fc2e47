#!/bin/bash
# Round 5 session 3: re-run the fixed GPU tests, the data-parallel gradient matrix (every gradient-routing feature,
# distinct per-rank batches), host decode cost on the box CPUs, prologue A/B for 1x1 consumers.
set -o pipefail
mkdir -p gpurun_out/r5
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -v -s --timeout 400 --timeout-method thread tests/test_fused_gpu.py tests/test_trajectory_inception_gpu.py tests/test_kernels_gpu.py -m gpu > gpurun_out/r5/r5_s3_pytest_fixed.log 2>&1
rc=$?; echo "fixed tests rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/r5/r5_s3_pytest_fixed.log | tail -5
case $rc in 0|1) ;; *) exit $rc ;; esac
DTM_DP_MATRIX=1 timeout -k 10 900 python -u -m pytest -v -s --timeout 300 --timeout-method thread tests/test_distributed.py -m gpu -k "step1_gradients" > gpurun_out/r5/r5_dp_matrix.log 2>&1
rc=$?; echo "dp matrix rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/r5/r5_dp_matrix.log | tail -5
case $rc in 0|1) ;; *) exit $rc ;; esac
timeout -k 10 200 python -u tools/decode_cpu_cost.py --images 512 > gpurun_out/r5/r5_decode_cpu_cost_box.log 2>&1; tail -8 gpurun_out/r5/r5_decode_cpu_cost_box.log
VARIANTS="base=;f1x1=prologue:fused1x1;nofdir=fdir:0" STEPS=6 ROUNDS=5 timeout -k 10 300 python -u tools/ab_step.py > gpurun_out/r5/r5_ab_prologue_1x1.log 2>&1; tail -3 gpurun_out/r5/r5_ab_prologue_1x1.log
echo done
