#!/bin/bash
# Round 5 session 50: split count (blocks per CU) of the register-staged weight-gradient tiles on Inception-v3's stem
# shapes (batch 128) and the 5x5 / small-K layers: WTILES=<tile>:<occ>.
set -o pipefail
mkdir -p gpurun_out/r5
export B=128 SET=custom WONLY=1 ROUNDS=3
export SHAPES_CUSTOM="149,32,32,3,3,1,VALID,1;147,32,64,3,3,1,SAME,1;35,48,64,5,5,1,SAME,3;35,288,64,1,1,1,SAME,9;35,288,48,1,1,1,SAME,3"
WTILES="6:2,6:3,6:6,6:8,6:12,1:2,1:3,1:6,1:8,1:12" timeout -k 10 300 python -u tools/conv_tile_sweep.py > gpurun_out/r5/r5_s50_wgrad_rs_occ_sweep.log 2>&1 || { tail -5 gpurun_out/r5/r5_s50_wgrad_rs_occ_sweep.log; exit 1; }
cat gpurun_out/r5/r5_s50_wgrad_rs_occ_sweep.log
echo done
