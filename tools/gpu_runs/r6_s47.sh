#!/bin/bash
# ResNet-50 dgrads with the act (BN-backward) epilogue after the 4-waves/SIMD register-staged tiles: policy vs tiles
set -o pipefail
mkdir -p gpurun_out/r6
ACT=1 ROUNDS=3 TILES=-1,3,4,21,26,40 timeout -k 10 600 python -u tools/conv_tile_sweep.py > gpurun_out/r6/r6_s47_act_resweep.log 2>&1 || exit 1
grep "dgact\|weighted" gpurun_out/r6/r6_s47_act_resweep.log
