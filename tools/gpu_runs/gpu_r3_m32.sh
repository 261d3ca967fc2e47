#!/bin/bash
# 32x32x16-MFMA conv tiles: numerics under the knob, per-shape A/B, whole-step A/B, bench.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_jpeg.py > gpurun_out/jpeg_tests.log 2>&1 || { echo "jpeg tests failed"; tail -40 gpurun_out/jpeg_tests.log; exit 1; }
tail -1 gpurun_out/jpeg_tests.log
DTM_MFMA32=1 timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_fused_gpu.py tests/test_fused_ops_gpu.py tests/test_zoo_gpu.py -m gpu > gpurun_out/m32_tests.log 2>&1 || { echo "m32 tests failed"; tail -40 gpurun_out/m32_tests.log; exit 1; }
tail -1 gpurun_out/m32_tests.log
timeout -k 10 300 python -u tools/mfma32_ab.py > gpurun_out/m32_shapes.log 2>&1 || { tail -30 gpurun_out/m32_shapes.log; exit 1; }
cat gpurun_out/m32_shapes.log
VARIANTS="m16=m32:0;m32=m32:1" ROUNDS=5 timeout -k 10 300 python -u tools/ab_step.py > gpurun_out/m32_step.log 2>&1 || { tail -30 gpurun_out/m32_step.log; exit 1; }
tail -2 gpurun_out/m32_step.log
