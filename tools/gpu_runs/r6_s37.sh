#!/bin/bash
# direct 3x3 weight gradient (conv3x3_wgrad_direct_kernel, wgrad tile 20): numerics + per-shape sweep
set -o pipefail
mkdir -p gpurun_out/r6
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -m gpu -k "wgrad" > gpurun_out/r6/r6_s37_pytest_wdirect.log 2>&1 || { tail -30 gpurun_out/r6/r6_s37_pytest_wdirect.log; exit 1; }
tail -1 gpurun_out/r6/r6_s37_pytest_wdirect.log
for o in 149_32_32_3 147_32_64_3; do
  SET=inception ONLY=$o WONLY=1 ROUNDS=3 B=128 WTILES=6:3,1:3,20:0 timeout -k 10 200 python -u tools/conv_tile_sweep.py >> gpurun_out/r6/r6_s37_wdirect_sweep.log 2>&1 || exit 1
  SET=inception ONLY=$o WONLY=1 WPRO=1 ROUNDS=3 B=128 WTILES=6:3,1:3,20:0 timeout -k 10 200 python -u tools/conv_tile_sweep.py >> gpurun_out/r6/r6_s37_wdirect_sweep.log 2>&1 || exit 1
done
for o in 56_64_64_3; do
  ONLY=$o WONLY=1 ROUNDS=3 WTILES=1:3,20:0 timeout -k 10 200 python -u tools/conv_tile_sweep.py >> gpurun_out/r6/r6_s37_wdirect_sweep.log 2>&1 || exit 1
  ONLY=$o WONLY=1 WPRO=1 ROUNDS=3 WTILES=1:3,20:0 timeout -k 10 200 python -u tools/conv_tile_sweep.py >> gpurun_out/r6/r6_s37_wdirect_sweep.log 2>&1 || exit 1
done
grep "wgrad " gpurun_out/r6/r6_s37_wdirect_sweep.log | grep -v weighted
