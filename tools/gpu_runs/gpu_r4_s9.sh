#!/bin/bash
# Round 4: merged sibling forward kernel vs per-member launches, sibling tests, default DP configs.
set -o pipefail
mkdir -p gpurun_out/r4
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "fwd_bn_multi" > gpurun_out/r4/pytest_fwdmulti.log 2>&1
echo "fwd_bn_multi tests rc=$?"; grep -E "PASS|FAIL|^E  " gpurun_out/r4/pytest_fwdmulti.log | cut -c1-200 | tail -14
timeout -k 10 300 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_fused_ops_gpu.py -k "sibling" > gpurun_out/r4/pytest_sibling.log 2>&1
echo "sibling tests rc=$?"; grep -E "PASS|FAIL|^E  " gpurun_out/r4/pytest_sibling.log | cut -c1-300 | tail -14
timeout -k 10 500 python -u -m pytest -v -s --timeout 450 --timeout-method thread tests/test_distributed.py -m gpu > gpurun_out/r4/pytest_dp_gpu.log 2>&1
echo "dp gpu tests rc=$?"; grep -E "PASSED|FAILED|^E  " gpurun_out/r4/pytest_dp_gpu.log | cut -c1-300 | tail -12
