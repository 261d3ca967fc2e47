#!/bin/bash
# Direct 3x3 kernel per-shape timing vs the implicit-GEMM tiles; stem wide-wgrad A/B.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for o in 56_64_64_3; do
TILES=-1,26,21,3 ROUNDS=3 ONLY=$o timeout -k 10 200 python -u tools/conv_tile_sweep.py > gpurun_out/sw_$o.log 2>&1 || { tail -20 gpurun_out/sw_$o.log; exit 1; }
grep -v amdgpu gpurun_out/sw_$o.log
done
for o in 149_32_32_3 147_32_64_3; do
SET=inception B=128 TILES=-1,26,32,21 ROUNDS=3 ONLY=$o timeout -k 10 200 python -u tools/conv_tile_sweep.py > gpurun_out/sw_$o.log 2>&1 || { tail -20 gpurun_out/sw_$o.log; exit 1; }
grep -v amdgpu gpurun_out/sw_$o.log
done
VARIANTS="w2=wwide:2;w0=wwide:0" ROUNDS=5 timeout -k 10 400 python -u tools/ab_step.py > gpurun_out/wwide2_rn.log 2>&1 || { tail -30 gpurun_out/wwide2_rn.log; exit 1; }
tail -3 gpurun_out/wwide2_rn.log
