#!/bin/bash
# Round 5 session 31: conv tile sweep over the Inception-v3 stem shapes (fwd+stats, act dgrad), incl. the direct 3x3 kernel.
set -o pipefail
mkdir -p gpurun_out/r5
export TMPDIR=/tmp
SET=custom B=128 STATS=1 ACT=1 ROUNDS=3 TILES=-1,0,3,4,21,24,26,32,40,60 SHAPES_CUSTOM="147,32,64,3,3,1,SAME,1;73,80,192,3,3,1,VALID,1;73,64,80,1,1,1,VALID,1;149,32,32,3,3,1,VALID,1" timeout -k 10 900 python -u tools/conv_tile_sweep.py > gpurun_out/r5/r5_s31_inception_stem_sweep.log 2>&1
rc=$?; grep -v amdgpu gpurun_out/r5/r5_s31_inception_stem_sweep.log | tail -30; exit $rc
