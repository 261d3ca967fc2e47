#!/bin/bash
# Round 4: ResNet-50 A/B after the split-store fix: merged projection-unit forward off, grouped strided-dgrad tile
# rule off.
set -o pipefail
mkdir -p gpurun_out/r4
export TMPDIR=/tmp
VARIANTS="base=;nofwd=sfwd:0;nodt=dtile:0" STEPS=8 ROUNDS=6 timeout -k 10 500 python -u tools/ab_step.py > gpurun_out/r4/ab_fwd_dtile_resnet.log 2>&1 || { tail -30 gpurun_out/r4/ab_fwd_dtile_resnet.log; exit 1; }
tail -4 gpurun_out/r4/ab_fwd_dtile_resnet.log
