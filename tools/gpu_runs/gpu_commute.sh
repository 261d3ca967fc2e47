#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_zoo_gpu.py tests/test_models.py -m gpu > gpurun_out/t_commute.log 2>&1 || { tail -40 gpurun_out/t_commute.log; exit 1; }
tail -2 gpurun_out/t_commute.log
MODEL=inception_v3_slim_old STEPS=15 ROUNDS=5 VARIANTS="commute=;orig=pcom:0" timeout -k 10 300 python -u tools/ab_step.py > gpurun_out/r2_ab_pool_commute_inception.log 2>&1 || { tail -20 gpurun_out/r2_ab_pool_commute_inception.log; exit 1; }
tail -2 gpurun_out/r2_ab_pool_commute_inception.log
