#!/bin/bash
# Inception-v3 stem dgrads with the BN backward epilogue (dgact): direct kernel (policy) vs the pipelined tiles
set -o pipefail
mkdir -p gpurun_out/r6
for o in 147_32_64_3 149_32_32_3; do
  SET=inception ONLY=$o ACT=1 ROUNDS=5 B=128 TILES=-1,60,26,32,21 timeout -k 10 200 python -u tools/conv_tile_sweep.py >> gpurun_out/r6/r6_s46_dgact_inception.log 2>&1 || exit 1
done
grep -v amdgpu gpurun_out/r6/r6_s46_dgact_inception.log
