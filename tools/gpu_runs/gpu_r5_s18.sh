#!/bin/bash
# Round 5 session 18: the distributed / engine GPU tests after removing the atomic act-sum path.
set -o pipefail
mkdir -p gpurun_out/r5
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_distributed.py tests/test_engine.py tests/test_kernels_gpu.py -m gpu > gpurun_out/r5/r5_s18_pytest.log 2>&1
rc=$?; grep -E "FAILED|ERROR" gpurun_out/r5/r5_s18_pytest.log | head -10; tail -1 gpurun_out/r5/r5_s18_pytest.log; exit $rc
