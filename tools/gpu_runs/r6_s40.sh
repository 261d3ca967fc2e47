#!/bin/bash
# Inception-v3: the stem's BN-fused weight gradient on the pipelined 64x256 tile (sbna, tuned on ResNet's 7x7 stem)
# vs the register-staged 32-row tile for its packed 3x3/2 3->32 stem conv
set -o pipefail
mkdir -p gpurun_out/r6
MODEL=inception_v3_slim_old VARIANTS="base=;nosbna=sbna:0" ROUNDS=5 timeout -k 10 500 python -u tools/ab_step.py > gpurun_out/r6/r6_s40_ab_sbna_inception.log 2>&1 || { tail -20 gpurun_out/r6/r6_s40_ab_sbna_inception.log; exit 1; }
tail -3 gpurun_out/r6/r6_s40_ab_sbna_inception.log
