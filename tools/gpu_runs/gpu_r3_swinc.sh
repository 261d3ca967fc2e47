#!/bin/bash
# Inception stem-region shapes: tile sweep (fwd / dgrad / wgrad) with the current kernels.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for o in 73_80_192_3 147_32_64_3 73_64_80_1; do
SET=inception B=128 TILES=-1,0,3,4,21,24,26,32,40 WTILES=-1,0,1,10,6 ROUNDS=3 ONLY=$o timeout -k 10 200 python -u tools/conv_tile_sweep.py > gpurun_out/swi_$o.log 2>&1 || { tail -20 gpurun_out/swi_$o.log; exit 1; }
grep -v amdgpu gpurun_out/swi_$o.log
done
