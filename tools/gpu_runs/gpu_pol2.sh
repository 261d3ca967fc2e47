#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > gpurun_out/t_pol2.log 2>&1 || { tail -40 gpurun_out/t_pol2.log; exit 1; }
tail -2 gpurun_out/t_pol2.log
MODEL=inception_v3_slim_old STEPS=15 ROUNDS=5 VARIANTS="pol2=;pol1=pol2:0" timeout -k 10 300 python -u tools/ab_step.py > gpurun_out/r2_ab_policy2_inception.log 2>&1 || { tail -20 gpurun_out/r2_ab_policy2_inception.log; exit 1; }
tail -2 gpurun_out/r2_ab_policy2_inception.log
VARIANTS="pol2=;pol1=pol2:0" timeout -k 10 300 python -u tools/ab_step.py > gpurun_out/r2_ab_policy2.log 2>&1 || { tail -20 gpurun_out/r2_ab_policy2.log; exit 1; }
tail -2 gpurun_out/r2_ab_policy2.log
