#!/bin/bash
# 4-wave 128x128-per-wave form of the 256x256 conv (tile 42) / wgrad (tile 17) tiles: numerics, per-shape sweep, step A/B
set -o pipefail
mkdir -p gpurun_out/r6
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -m gpu -k "pipelined_tiles or act_dgrad_tiles" > gpurun_out/r6/r6_s27_pytest_w4.log 2>&1 || { tail -30 gpurun_out/r6/r6_s27_pytest_w4.log; exit 1; }
tail -1 gpurun_out/r6/r6_s27_pytest_w4.log
ROUNDS=5 TILES=40,42 STATS=1 ACT=1 WGRAD= WTILES=12:1,17:1 timeout -k 10 400 python -u tools/conv_tile_sweep.py > gpurun_out/r6/r6_s27_sweep_w4.log 2>&1 || { tail -20 gpurun_out/r6/r6_s27_sweep_w4.log; exit 1; }
grep -v amdgpu gpurun_out/r6/r6_s27_sweep_w4.log | tail -40
VARIANTS="base=;w4=w4:1" ROUNDS=4 timeout -k 10 400 python -u tools/ab_step.py > gpurun_out/r6/r6_s27_ab_w4.log 2>&1 || { tail -20 gpurun_out/r6/r6_s27_ab_w4.log; exit 1; }
tail -3 gpurun_out/r6/r6_s27_ab_w4.log
