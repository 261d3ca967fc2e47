#!/bin/bash
# Round 4: DP gradient matrix (1 vs 2 gloo ranks on the HIP kernels) + BN moving statistics across ranks with
# different batches (tests/test_distributed.py -m gpu); workers print a line per step (-s).
set -o pipefail
mkdir -p gpurun_out/r4
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_fused_ops_gpu.py -k "sibling" > gpurun_out/r4/pytest_sibling.log 2>&1
echo "sibling tests rc=$?"; grep -E "PASS|FAIL|ERROR" gpurun_out/r4/pytest_sibling.log | cut -c1-160 | tail -8
timeout -k 10 300 python -u tools/dp_grad_diag.py resnet_v1_50 DTM_WGRAD_STREAM=0 > gpurun_out/r4/diag_resnet_wgs0.log 2>&1
echo "diag resnet wgs0 rc=$?"; grep -E "RESULT|tensors differ|Error|error" gpurun_out/r4/diag_resnet_wgs0.log | head -5
timeout -k 10 1000 python -u -m pytest -v -s --timeout 300 --timeout-method thread tests/test_distributed.py -m gpu > gpurun_out/r4/pytest_dp_gpu.log 2>&1
echo "dp gpu tests rc=$?"; grep -E "PASS|FAIL|ERROR" gpurun_out/r4/pytest_dp_gpu.log | cut -c1-160 | tail -20
