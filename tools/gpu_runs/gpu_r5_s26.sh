#!/bin/bash
# Round 5 session 26: the conv / wgrad tile decisions of one Inception-v3 training step (DTM_TILE_LOG=1).
set -o pipefail
mkdir -p gpurun_out/r5
export TMPDIR=/tmp
DTM_TILE_LOG=1 timeout -k 10 300 python -u bench.py --model inception_v3_slim_old --graph 0 --steps 1 --warmup 1 > gpurun_out/r5/r5_s26_tile_log_inception.log 2>&1
rc=$?; grep -c dtm_wgrad gpurun_out/r5/r5_s26_tile_log_inception.log; exit $rc
