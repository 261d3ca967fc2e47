#!/bin/bash
# High-priority main stream vs default (side-stream weight gradients on).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "device_state" > gpurun_out/prio_tests.log 2>&1 || { tail -30 gpurun_out/prio_tests.log; exit 1; }
tail -1 gpurun_out/prio_tests.log
VARIANTS="base=;prio=prio:1" ROUNDS=5 timeout -k 10 400 python -u tools/ab_step.py > gpurun_out/prio_step.log 2>&1 || { tail -30 gpurun_out/prio_step.log; exit 1; }
tail -3 gpurun_out/prio_step.log
