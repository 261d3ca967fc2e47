#!/bin/bash
# Round 6 session 13: ResNet-50 teacher-forced per-segment check (masked unit input gradients), final_loss spread log.
set -o pipefail
mkdir -p gpurun_out/r6
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 500 --timeout-method thread tests/test_trajectory_resnet_gpu.py -m gpu -k teacher > gpurun_out/r6/r6_s13_pytest_resnet.log 2>&1 || { tail -40 gpurun_out/r6/r6_s13_pytest_resnet.log; exit 1; }
grep -E "tensors|passed|failed" gpurun_out/r6/r6_s13_pytest_resnet.log | tail -4
timeout -k 10 500 python -u tools/loss_spread.py > gpurun_out/r6/r6_s13_loss_spread.log 2>&1 || { tail -20 gpurun_out/r6/r6_s13_loss_spread.log; exit 1; }
cat gpurun_out/r6/r6_s13_loss_spread.log
