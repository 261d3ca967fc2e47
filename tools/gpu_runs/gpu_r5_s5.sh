#!/bin/bash
# Round 5 session 5: 3-slot 8-wave tiles (41: 256x128, 42: 128x256, 144 KiB LDS) vs the policy and the 2-slot 256x256.
set -o pipefail
mkdir -p gpurun_out/r5
export TMPDIR=/tmp
STATS=1 ACT=1 TILES=-1,40,41,42,21 ROUNDS=3 timeout -k 10 600 python -u tools/conv_tile_sweep.py > gpurun_out/r5/r5_tile_sweep_w8ns3.log 2>&1
rc=$?; tail -2 gpurun_out/r5/r5_tile_sweep_w8ns3.log; exit $rc
