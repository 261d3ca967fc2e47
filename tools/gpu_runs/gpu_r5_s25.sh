#!/bin/bash
# Round 5 session 25: wgrad tiles for the <= 64-channel Inception-v3 layers (register-staged 1 / 6 vs pipelined 10 / 11).
set -o pipefail
mkdir -p gpurun_out/r5
export TMPDIR=/tmp
SET=inception B=128 WTILES=1:0,6:0,10:0,11:0 WONLY=1 ROUNDS=3 timeout -k 10 400 python -u tools/conv_tile_sweep.py > gpurun_out/r5/r5_s25_wgrad_small_k_sweep.log 2>&1
rc=$?; grep -v amdgpu gpurun_out/r5/r5_s25_wgrad_small_k_sweep.log | tail -30; exit $rc
