#!/bin/bash
# Inception-v3 step: direct 3x3 kernel with 32-channel output tiles for the stem's 32->64 conv (ct32) vs 64-channel
set -o pipefail
mkdir -p gpurun_out/r6
MODEL=inception_v3_slim_old VARIANTS="base=;ct32=ct32:1" ROUNDS=5 timeout -k 10 500 python -u tools/ab_step.py > gpurun_out/r6/r6_s30_ab_ct32_inception.log 2>&1 || { tail -20 gpurun_out/r6/r6_s30_ab_ct32_inception.log; exit 1; }
tail -3 gpurun_out/r6/r6_s30_ab_ct32_inception.log
