#!/bin/bash
# fp32-atomic split-K weight gradients vs slabs + reduce: numerics (all wgrad tests) and step A/B (Inception, ResNet).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
DTM_WGRAD_ATOMIC=64 timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_fused_ops_gpu.py tests/test_fused_gpu.py -k "wgrad or conv or stem" > gpurun_out/watom_tests.log 2>&1 || { tail -30 gpurun_out/watom_tests.log; exit 1; }
tail -1 gpurun_out/watom_tests.log
MODEL=inception_v3_slim_old VARIANTS="slab=watom:0;a16=watom:16;a64=watom:64;a512=watom:512" ROUNDS=4 timeout -k 10 400 python -u tools/ab_step.py > gpurun_out/watom_inc.log 2>&1 || { tail -30 gpurun_out/watom_inc.log; exit 1; }
tail -4 gpurun_out/watom_inc.log
VARIANTS="slab=watom:0;a16=watom:16;a64=watom:64;a512=watom:512" ROUNDS=4 timeout -k 10 400 python -u tools/ab_step.py > gpurun_out/watom_rn.log 2>&1 || { tail -30 gpurun_out/watom_rn.log; exit 1; }
tail -4 gpurun_out/watom_rn.log
