#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "pipelined or wgrad" -m gpu > gpurun_out/t_k32.log 2>&1 || { tail -40 gpurun_out/t_k32.log; exit 1; }
tail -2 gpurun_out/t_k32.log
SET=inception B=128 ONLY=_32_ TILES=-1,26 WTILES=-1,1,6 ROUNDS=3 timeout -k 10 300 python -u tools/conv_tile_sweep.py > gpurun_out/r2_sweep_k32.log 2>&1 || { tail -20 gpurun_out/r2_sweep_k32.log; exit 1; }
grep -v "^/opt" gpurun_out/r2_sweep_k32.log
MODEL=inception_v3_slim_old STEPS=15 ROUNDS=5 VARIANTS="k32=;k64=k32:0" timeout -k 10 300 python -u tools/ab_step.py > gpurun_out/r2_ab_k32_inception.log 2>&1 || { tail -20 gpurun_out/r2_ab_k32_inception.log; exit 1; }
tail -2 gpurun_out/r2_ab_k32_inception.log
