#!/bin/bash
# Sibling-merge / act hand-off GPU tests only.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_fused_ops_gpu.py -k "sibling or handoff or chain" > gpurun_out/sibtest.log 2>&1; rc=$?
grep -E "Error|assert|passed|failed" gpurun_out/sibtest.log | head -30
exit $rc
