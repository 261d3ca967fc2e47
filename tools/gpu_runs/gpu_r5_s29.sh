#!/bin/bash
# Round 5 session 29: conv_nt tile sweep over the Inception-v3 step's most frequent shapes (fwd+stats, act dgrad).
set -o pipefail
mkdir -p gpurun_out/r5
export TMPDIR=/tmp
SET=custom B=128 STATS=1 ACT=1 ROUNDS=3 TILES=-1,0,4,21,24,26,40 SHAPES_CUSTOM="17,192,192,7,1,1,SAME,4;17,192,192,1,7,1,SAME,4;17,160,160,7,1,1,SAME,4;17,160,160,1,7,1,SAME,4;17,160,192,7,1,1,SAME,2;17,128,128,7,1,1,SAME,2;35,64,96,3,3,1,SAME,4;35,96,96,3,3,1,SAME,3;35,48,64,5,5,1,SAME,3;8,384,384,3,1,1,SAME,4;8,448,384,3,3,1,SAME,2" timeout -k 10 900 python -u tools/conv_tile_sweep.py > gpurun_out/r5/r5_s29_inception_tile_sweep.log 2>&1
rc=$?; grep -v amdgpu gpurun_out/r5/r5_s29_inception_tile_sweep.log | tail -60; exit $rc
