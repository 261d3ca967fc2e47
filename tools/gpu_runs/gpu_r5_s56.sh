#!/bin/bash
# Round 5 session 56: ResNet-50 same-process A/B of the remaining launch-policy knobs under this round's kernels
# (tools/ab_step.py: cpt, ntld, sc, red, few, kwide, k32).
set -o pipefail
mkdir -p gpurun_out/r5
VARIANTS="base=;cpt4=cpt:4;cpt16=cpt:16;ntld0=ntld:0;ntld1=ntld:1;ntld2=ntld:2" ROUNDS=5 STEPS=6 timeout -k 10 400 python -u tools/ab_step.py > gpurun_out/r5/r5_s56_ab_a.log 2>&1 || { tail -5 gpurun_out/r5/r5_s56_ab_a.log; exit 1; }
tail -6 gpurun_out/r5/r5_s56_ab_a.log
VARIANTS="base=;sc4=sc:4:4096;sc6=sc:6:4096;sc5k2=sc:5:2048;sc5k8=sc:5:8192;red32=red:0:32:0;red128=red:0:128:0" ROUNDS=5 STEPS=6 timeout -k 10 400 python -u tools/ab_step.py > gpurun_out/r5/r5_s56_ab_b.log 2>&1 || { tail -5 gpurun_out/r5/r5_s56_ab_b.log; exit 1; }
tail -7 gpurun_out/r5/r5_s56_ab_b.log
VARIANTS="base=;few0=few:0;kwide0=kwide:0;k32off=k32:0;fdir0=fdir:0" ROUNDS=5 STEPS=6 timeout -k 10 400 python -u tools/ab_step.py > gpurun_out/r5/r5_s56_ab_c.log 2>&1 || { tail -5 gpurun_out/r5/r5_s56_ab_c.log; exit 1; }
tail -5 gpurun_out/r5/r5_s56_ab_c.log
echo done
