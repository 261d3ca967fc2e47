#!/bin/bash
# hipGraph-captured step with the side-stream weight gradients (DTM_WGRAD_STREAM_GRAPH=1) vs single-stream capture
# vs eager, Inception-v3 and ResNet-50 (same-process A/B, interleaved rounds).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
export DTM_WGRAD_STREAM_GRAPH=1
MODEL=inception_v3_slim_old GRAPH=1 VARIANTS="g1=wgs:0;gside=wgs:1" ROUNDS=6 timeout -k 10 400 python -u tools/ab_step.py > gpurun_out/graphside_inc.log 2>&1 || { tail -30 gpurun_out/graphside_inc.log; exit 1; }
tail -3 gpurun_out/graphside_inc.log
MODEL=resnet_v1_50 GRAPH=1 VARIANTS="g1=wgs:0;gside=wgs:1" ROUNDS=5 timeout -k 10 400 python -u tools/ab_step.py > gpurun_out/graphside_rn.log 2>&1 || { tail -30 gpurun_out/graphside_rn.log; exit 1; }
tail -3 gpurun_out/graphside_rn.log
MODEL=resnet_v1_50 VARIANTS="eside=wgs:1" ROUNDS=5 timeout -k 10 400 python -u tools/ab_step.py > gpurun_out/graphside_rn_eager.log 2>&1 || { tail -30 gpurun_out/graphside_rn_eager.log; exit 1; }
tail -2 gpurun_out/graphside_rn_eager.log
