#!/bin/bash
# Round-4 final evidence C: the zoo GPU tests (their MIOpen-based references now on the CPU), then smoke + benches.
set -o pipefail
mkdir -p gpurun_out/r4
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_zoo_gpu.py -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r4/r4_final_pytest_zoo.log 2>&1
rc=$?; echo "zoo suite rc=$rc"; grep -E "FAILED|ERROR" gpurun_out/r4/r4_final_pytest_zoo.log | head -10; tail -1 gpurun_out/r4/r4_final_pytest_zoo.log
if [ $rc -ne 0 ]; then exit $rc; fi
bash tools/gpu_runs/gpu_r4_finalB.sh
