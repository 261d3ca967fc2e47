#!/bin/bash
# Round 6 session 9: stem weight-gradient tiles (64x256 register-staged 7 / 8 vs the policy's 64x128), with the fused
# BN backward as training runs it.
set -o pipefail
mkdir -p gpurun_out/r6
TILES=-1 WTILES="-1,1,1:2,7,7:1,7:2,7:3,8,8:1,8:2" ROUNDS=5 timeout -k 10 300 python -u tools/stem_sweep.py > gpurun_out/r6/r6_s9_stem_wgrad.log 2>&1 || { tail -20 gpurun_out/r6/r6_s9_stem_wgrad.log; exit 1; }
cat gpurun_out/r6/r6_s9_stem_wgrad.log
