#!/bin/bash
# Round 5 session 4: re-sweep every ResNet-50 conv shape over the conv tiles (forward with statistics, dgrad with the
# act epilogue) with the round-4/5 kernels, to find stale shape-policy picks.
set -o pipefail
mkdir -p gpurun_out/r5
export TMPDIR=/tmp
STATS=1 ACT=1 TILES=-1,0,3,4,21,24,26,40 ROUNDS=3 timeout -k 10 900 python -u tools/conv_tile_sweep.py > gpurun_out/r5/r5_tile_resweep_resnet.log 2>&1
rc=$?; tail -3 gpurun_out/r5/r5_tile_resweep_resnet.log; exit $rc
