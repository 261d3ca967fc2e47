#!/bin/bash
# Inception-v3 stem weight gradients (147/149 maps, 32/64 channels): register-staged tiles vs pipelined, with and
# without the x prologue
set -o pipefail
mkdir -p gpurun_out/r6
for o in 149_32_32_3 147_32_64_3 73_64_80_1; do
  SET=inception ONLY=$o WONLY=1 ROUNDS=3 B=128 WTILES=6:3,1:3,0:3,7:3,11:2,10:2 timeout -k 10 200 python -u tools/conv_tile_sweep.py >> gpurun_out/r6/r6_s31_stem_wgrad_inception.log 2>&1 || exit 1
  SET=inception ONLY=$o WONLY=1 WPRO=1 ROUNDS=3 B=128 WTILES=6:3,1:3,0:3 timeout -k 10 200 python -u tools/conv_tile_sweep.py >> gpurun_out/r6/r6_s31_stem_wgrad_inception.log 2>&1 || exit 1
done
grep "wgrad " gpurun_out/r6/r6_s31_stem_wgrad_inception.log
