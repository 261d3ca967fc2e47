#!/bin/bash
# Inception stem direct 3x3 kernels: 32-channel output tiles for K = 64 (occupancy) vs the 64-channel tile
set -o pipefail
mkdir -p gpurun_out/r6
for ct in 0 1; do
  echo "== DTM_DIRECT_CT32=$ct" >> gpurun_out/r6/r6_s29_direct_ct32.log
  DTM_DIRECT_CT32=$ct SET=inception ONLY=147_32_64_3 ACT=1 ROUNDS=5 TILES=-1 B=128 timeout -k 10 200 python -u tools/conv_tile_sweep.py >> gpurun_out/r6/r6_s29_direct_ct32.log 2>&1 || exit 1
  DTM_DIRECT_CT32=$ct SET=inception ONLY=149_32_32_3 ACT=1 ROUNDS=5 TILES=-1 B=128 timeout -k 10 200 python -u tools/conv_tile_sweep.py >> gpurun_out/r6/r6_s29_direct_ct32.log 2>&1 || exit 1
done
grep -v amdgpu gpurun_out/r6/r6_s29_direct_ct32.log
