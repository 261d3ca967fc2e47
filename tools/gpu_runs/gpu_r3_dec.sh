#!/bin/bash
# Strided-dgrad tile sweep (decomposed path) + step timeline with the side stream.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TILES=-1,0,3,4,21,24,26,40 ROUNDS=3 timeout -k 10 400 python -u tools/conv_tile_sweep.py > gpurun_out/sweep_dec.log 2>&1 || { tail -30 gpurun_out/sweep_dec.log; exit 1; }
grep -E "s2|shape|total" gpurun_out/sweep_dec.log
bash tools/gpu_runs/gpu_r3_tl.sh
