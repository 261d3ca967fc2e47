#!/bin/bash
# Round 4: DP gradient matrix (1 vs 2 gloo ranks on the HIP kernels) + BN moving statistics across ranks with
# different batches (tests/test_distributed.py -m gpu).
set -o pipefail
mkdir -p gpurun_out/r4
export TMPDIR=/tmp
timeout -k 10 1050 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_distributed.py -m gpu > gpurun_out/r4/pytest_dp_gpu.log 2>&1
echo "dp gpu tests rc=$?"; grep -E "PASS|FAIL|ERROR" gpurun_out/r4/pytest_dp_gpu.log | cut -c1-160 | tail -20
