#!/bin/bash
# Round 5 session 23: Inception-v3 BN-apply prologue policy A/B (materialise vs prologue for spatial / all consumers).
set -o pipefail
mkdir -p gpurun_out/r5
export TMPDIR=/tmp
MODEL=inception_v3_slim_old STEPS=6 ROUNDS=4 VARIANTS="base=;spatial=prologue:spatial;fused=prologue:fused" timeout -k 10 600 python -u tools/ab_step.py > gpurun_out/r5/r5_s23_ab_prologue_inception.log 2>&1
rc=$?; tail -5 gpurun_out/r5/r5_s23_ab_prologue_inception.log; exit $rc
