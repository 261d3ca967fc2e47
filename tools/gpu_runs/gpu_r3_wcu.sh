#!/bin/bash
# Split-K sizing of the main-stream / stem weight gradients (percent of the CUs the split policy fills), ResNet-50 and
# Inception-v3 (eager A/B), + side-stream fraction fine sweep.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
VARIANTS="base=;swc50=swc:50;swc200=swc:200;swc300=swc:300;scu65=scu:65;scu85=scu:85" ROUNDS=5 timeout -k 10 500 python -u tools/ab_step.py > gpurun_out/r3_ab_wgrad_cus_resnet.log 2>&1 || { tail -30 gpurun_out/r3_ab_wgrad_cus_resnet.log; exit 1; }
tail -6 gpurun_out/r3_ab_wgrad_cus_resnet.log
MODEL=inception_v3_slim_old VARIANTS="base=;wcu50=wcu:50;wcu75=wcu:75;wcu150=wcu:150;wcu200=wcu:200" ROUNDS=5 timeout -k 10 500 python -u tools/ab_step.py > gpurun_out/r3_ab_wgrad_cus_inception.log 2>&1 || { tail -30 gpurun_out/r3_ab_wgrad_cus_inception.log; exit 1; }
tail -5 gpurun_out/r3_ab_wgrad_cus_inception.log
