#!/bin/bash
# Round 4: ResNet-50 merged projection-unit forward again, now that merged-head convs take the 128x128 tile.
set -o pipefail
mkdir -p gpurun_out/r4
export TMPDIR=/tmp
VARIANTS="base=;rfwd=rfwd:1" STEPS=8 ROUNDS=6 timeout -k 10 400 python -u tools/ab_step.py > gpurun_out/r4/ab_rfwd_resnet.log 2>&1 || { tail -30 gpurun_out/r4/ab_rfwd_resnet.log; exit 1; }
tail -3 gpurun_out/r4/ab_rfwd_resnet.log
