#!/bin/bash
# Round 5 session 55: ResNet-50 same-process A/B of the side-stream weight gradients' split-K CU fraction (scu) and the
# stem weight gradient's CU share (swc), re-tuned under this round's kernels (round 3 picked scu 75).
set -o pipefail
mkdir -p gpurun_out/r5
VARIANTS="base=;scu50=scu:50;scu60=scu:60;scu90=scu:90;scu100=scu:100" ROUNDS=5 STEPS=6 timeout -k 10 400 python -u tools/ab_step.py > gpurun_out/r5/r5_s55_ab_scu_resnet.log 2>&1 || { tail -5 gpurun_out/r5/r5_s55_ab_scu_resnet.log; exit 1; }
tail -5 gpurun_out/r5/r5_s55_ab_scu_resnet.log
VARIANTS="base=;swc75=swc:75;swc50=swc:50;wcu90=wcu:90" ROUNDS=5 STEPS=6 timeout -k 10 400 python -u tools/ab_step.py > gpurun_out/r5/r5_s55_ab_swc_resnet.log 2>&1 || { tail -5 gpurun_out/r5/r5_s55_ab_swc_resnet.log; exit 1; }
tail -4 gpurun_out/r5/r5_s55_ab_swc_resnet.log
echo done
