#!/bin/bash
# Round 6 session 5: block-output dgrad tiles vs their HBM floor.
set -o pipefail
mkdir -p gpurun_out/r6
TILES=-1,4,3,0,40,21,24,26 timeout -k 10 300 python -u tools/act_dgrad_bench.py > gpurun_out/r6/r6_s5_act_dgrad.log 2>&1 || { tail -20 gpurun_out/r6/r6_s5_act_dgrad.log; exit 1; }
cat gpurun_out/r6/r6_s5_act_dgrad.log
