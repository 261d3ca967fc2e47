#!/bin/bash
# stage-1 K=64 weight gradients (ResNet-50 56x56 conv1 1x1 256->64 and conv2 3x3 64->64): register-staged 64x128
# (tile 1) vs the pipelined 64x256 (11) / 128x128 (10), without and with the BN-apply prologue on x
set -o pipefail
mkdir -p gpurun_out/r6
for o in 56_256_64_1 56_64_64_3; do
  ONLY=$o WONLY=1 ROUNDS=5 WTILES=1:3,1:2,11:1,11:2,11:3,10:2 timeout -k 10 200 python -u tools/conv_tile_sweep.py >> gpurun_out/r6/r6_s26_wgrad_k64.log 2>&1 || exit 1
  ONLY=$o WONLY=1 WPRO=1 ROUNDS=5 WTILES=1:3,1:2,0:3 timeout -k 10 200 python -u tools/conv_tile_sweep.py >> gpurun_out/r6/r6_s26_wgrad_k64.log 2>&1 || exit 1
done
