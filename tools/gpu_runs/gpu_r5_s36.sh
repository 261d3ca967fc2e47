#!/bin/bash
# Round 5 session 36: ResNet-50 stem forward / weight-gradient tile sweep with this round's kernels.
set -o pipefail
mkdir -p gpurun_out/r5
export TMPDIR=/tmp
TILES=-1,0,3,4,21,24,26 WTILES=-1,0,1,10,11,12:1 ROUNDS=3 timeout -k 10 400 python -u tools/stem_sweep.py > gpurun_out/r5/r5_s36_stem_sweep.log 2>&1
rc=$?; grep -v amdgpu gpurun_out/r5/r5_s36_stem_sweep.log; exit $rc
