#!/bin/bash
# Round-4 final evidence A: the whole GPU suite.
set -o pipefail
mkdir -p gpurun_out/r4
export TMPDIR=/tmp
timeout -k 10 1080 python -u -m pytest tests -m gpu -v --timeout 450 --timeout-method thread > gpurun_out/r4/r4_final_pytest_gpu.log 2>&1
rc=$?; echo "gpu suite rc=$rc"; grep -E "FAILED|ERROR" gpurun_out/r4/r4_final_pytest_gpu.log | head -10; tail -1 gpurun_out/r4/r4_final_pytest_gpu.log
exit $rc
