#!/bin/bash
# Round 5 session 57: confirmation A/B of the stats-combine grid cap 8192 (sc:5:8192) vs 4096 on ResNet-50 and Inception-v3.
set -o pipefail
mkdir -p gpurun_out/r5
VARIANTS="base=;sc5k8=sc:5:8192;sc5k6=sc:5:6144" ROUNDS=8 STEPS=6 timeout -k 10 400 python -u tools/ab_step.py > gpurun_out/r5/r5_s57_ab_sc_resnet.log 2>&1 || { tail -5 gpurun_out/r5/r5_s57_ab_sc_resnet.log; exit 1; }
tail -3 gpurun_out/r5/r5_s57_ab_sc_resnet.log
MODEL=inception_v3_slim_old VARIANTS="base=;sc5k8=sc:5:8192;sc5k6=sc:5:6144" ROUNDS=6 STEPS=6 timeout -k 10 400 python -u tools/ab_step.py > gpurun_out/r5/r5_s57_ab_sc_inception.log 2>&1 || { tail -5 gpurun_out/r5/r5_s57_ab_sc_inception.log; exit 1; }
tail -3 gpurun_out/r5/r5_s57_ab_sc_inception.log
echo done
