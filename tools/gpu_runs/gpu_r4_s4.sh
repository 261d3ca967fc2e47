#!/bin/bash
# Round 4: sibling numerics (merged forward / grouped combine), the DP gradient matrix (1 vs 2 gloo ranks, every
# config in one process per rank) + BN moving statistics across ranks with different batches; workers print per step.
set -o pipefail
mkdir -p gpurun_out/r4
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_fused_ops_gpu.py -k "sibling" > gpurun_out/r4/pytest_sibling.log 2>&1
echo "sibling tests rc=$?"; grep -E "PASS|FAIL|ERROR" gpurun_out/r4/pytest_sibling.log | cut -c1-160 | tail -10
timeout -k 10 700 python -u -m pytest -v -s --timeout 600 --timeout-method thread tests/test_distributed.py -m gpu > gpurun_out/r4/pytest_dp_gpu.log 2>&1
echo "dp gpu tests rc=$?"; grep -E "PASS|FAIL|ERROR|assert" gpurun_out/r4/pytest_dp_gpu.log | cut -c1-300 | tail -12
