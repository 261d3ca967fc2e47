#!/bin/bash
# Inception-v3's packed stem (3x3/2 3->32) weight gradient with the fused BN backward: the policy's tile (15 since the
# ResNet stem rule) vs the register-staged 32-row tile 6 and others
set -o pipefail
mkdir -p gpurun_out/r6
INC=1 TILES=-1 WTILES=-1,6,1,7,15:2,14:1 ROUNDS=5 timeout -k 10 300 python -u tools/stem_sweep.py > gpurun_out/r6/r6_s41_stem_inception.log 2>&1 || { tail -20 gpurun_out/r6/r6_s41_stem_inception.log; exit 1; }
grep -v amdgpu gpurun_out/r6/r6_s41_stem_inception.log
