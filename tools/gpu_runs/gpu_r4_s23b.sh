#!/bin/bash
# Round 4: ResNet-50 side-stream split-K CU fraction re-check after this round's changes.
set -o pipefail
mkdir -p gpurun_out/r4
export TMPDIR=/tmp
VARIANTS="base=;s60=scu:60;s90=scu:90" STEPS=8 ROUNDS=6 timeout -k 10 450 python -u tools/ab_step.py > gpurun_out/r4/ab_scu_resnet.log 2>&1 || { tail -30 gpurun_out/r4/ab_scu_resnet.log; exit 1; }
tail -4 gpurun_out/r4/ab_scu_resnet.log
