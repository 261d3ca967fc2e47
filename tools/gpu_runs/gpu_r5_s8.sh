#!/bin/bash
# Round 5 session 8: the BSP collectives over RCCL at one rank (forced), and the rest of the distributed GPU tests.
set -o pipefail
mkdir -p gpurun_out/r5
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -v -s --timeout 300 --timeout-method thread tests/test_distributed.py -m gpu > gpurun_out/r5/r5_s8_pytest_dist.log 2>&1
rc=$?; echo "rc=$rc"; grep -E "PASSED|FAILED|ERROR" gpurun_out/r5/r5_s8_pytest_dist.log | head -20; tail -1 gpurun_out/r5/r5_s8_pytest_dist.log
exit $rc
