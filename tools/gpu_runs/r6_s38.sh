#!/bin/bash
# ResNet-50 56x56 3x3 64->64: the direct 3x3 kernel (tile 60, 32-channel output tiles) vs the policy's tiles
set -o pipefail
mkdir -p gpurun_out/r6
ONLY=56_64_64_3 ACT=1 ROUNDS=5 TILES=-1,60,26 timeout -k 10 200 python -u tools/conv_tile_sweep.py > gpurun_out/r6/r6_s38_direct_resnet.log 2>&1 || exit 1
grep -v amdgpu gpurun_out/r6/r6_s38_direct_resnet.log
