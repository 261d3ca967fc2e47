#!/bin/bash
# Round 6 session 12: stem BN-fused wgrad tile (numerics + step A/B), ResNet-50 production-shape determinism and the
# teacher-forced per-segment check, the final_loss spread log.
set -o pipefail
mkdir -p gpurun_out/r6
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_fused_ops_gpu.py -m gpu -k "stem" > gpurun_out/r6/r6_s12_pytest_stem.log 2>&1 || { tail -30 gpurun_out/r6/r6_s12_pytest_stem.log; exit 1; }
tail -1 gpurun_out/r6/r6_s12_pytest_stem.log
VARIANTS="sbna=;old=sbna:0" ROUNDS=5 timeout -k 10 300 python -u tools/ab_step.py > gpurun_out/r6/r6_s12_ab_sbna.log 2>&1 || { tail -20 gpurun_out/r6/r6_s12_ab_sbna.log; exit 1; }
tail -2 gpurun_out/r6/r6_s12_ab_sbna.log
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 500 --timeout-method thread tests/test_trajectory_resnet_gpu.py -m gpu > gpurun_out/r6/r6_s12_pytest_resnet.log 2>&1 || { tail -40 gpurun_out/r6/r6_s12_pytest_resnet.log; exit 1; }
grep -E "tensors|PASS|FAIL|passed|failed" gpurun_out/r6/r6_s12_pytest_resnet.log | tail -8
timeout -k 10 400 python -u tools/loss_spread.py > gpurun_out/r6/r6_s12_loss_spread.log 2>&1 || { tail -20 gpurun_out/r6/r6_s12_loss_spread.log; exit 1; }
cat gpurun_out/r6/r6_s12_loss_spread.log
