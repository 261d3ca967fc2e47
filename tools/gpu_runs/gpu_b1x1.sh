#!/bin/bash
# one-pass 1x1 conv+BN backward: numerics tests, whole-net gradient checks, same-process A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_fused_ops_gpu.py -k "one_pass or block_output or stem" > gpurun_out/t_b1x1.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/t_b1x1.log; exit 1; }
grep -E "passed|failed" gpurun_out/t_b1x1.log | tail -3
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_trajectory_gpu.py tests/test_fused_gpu.py > gpurun_out/t_b1x1_net.log 2>&1 || { echo "net tests failed"; tail -40 gpurun_out/t_b1x1_net.log; exit 1; }
tail -2 gpurun_out/t_b1x1_net.log
VARIANTS="${VARIANTS:-fused=;off=b1x1:0}" ROUNDS=5 timeout -k 10 300 python tools/ab_step.py > gpurun_out/ab_b1x1.log 2>&1 || { tail -20 gpurun_out/ab_b1x1.log; exit 1; }
tail -3 gpurun_out/ab_b1x1.log
