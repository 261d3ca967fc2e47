#!/bin/bash
# Round 4: ResNet-50 same-process A/B of this round's default-on changes (merged projection-unit forward, grouped
# sibling combine, LPT strided-dgrad order, sibling merge itself) + bench.
set -o pipefail
mkdir -p gpurun_out/r4
export TMPDIR=/tmp
VARIANTS="base=;nofwd=sfwd:0;nocomb=scomb:0;nolpt=lpt:0;nosib=sib:0,ahand:0" STEPS=6 ROUNDS=5 timeout -k 10 500 python -u tools/ab_step.py > gpurun_out/r4/ab_r4knobs_resnet.log 2>&1 || { tail -30 gpurun_out/r4/ab_r4knobs_resnet.log; exit 1; }
tail -5 gpurun_out/r4/ab_r4knobs_resnet.log
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r4/bench_resnet_s10.log 2>&1 || { tail -30 gpurun_out/r4/bench_resnet_s10.log; exit 1; }
tail -1 gpurun_out/r4/bench_resnet_s10.log | cut -c1-200
MODEL=inception_v3_slim_old VARIANTS="base=;nocomb=scomb:0;nolpt=lpt:0" STEPS=6 ROUNDS=5 timeout -k 10 400 python -u tools/ab_step.py > gpurun_out/r4/ab_r4knobs_inception.log 2>&1 || { tail -30 gpurun_out/r4/ab_r4knobs_inception.log; exit 1; }
tail -3 gpurun_out/r4/ab_r4knobs_inception.log
