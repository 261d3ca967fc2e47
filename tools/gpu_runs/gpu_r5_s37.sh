#!/bin/bash
# Round 5 session 37: split-K sizing (blocks per CU the split count targets) of the Inception-v3 17x17 / 35x35 wgrads.
set -o pipefail
mkdir -p gpurun_out/r5
export TMPDIR=/tmp
SET=custom B=128 WTILES=10:1,10:2,10:3,10:4,12:1 WONLY=1 ROUNDS=3 SHAPES_CUSTOM="17,160,160,7,1,1,SAME,8;17,160,160,1,7,1,SAME,8;17,192,192,7,1,1,SAME,8;17,160,192,7,1,1,SAME,4;17,128,128,7,1,1,SAME,4;35,64,96,3,3,1,SAME,4;35,96,96,3,3,1,SAME,3;8,384,384,3,1,1,SAME,8;17,768,704,1,1,1,SAME,2" timeout -k 10 400 python -u tools/conv_tile_sweep.py > gpurun_out/r5/r5_s37_wgrad_occ_sweep.log 2>&1
rc=$?; grep -v amdgpu gpurun_out/r5/r5_s37_wgrad_occ_sweep.log | tail -14; exit $rc
