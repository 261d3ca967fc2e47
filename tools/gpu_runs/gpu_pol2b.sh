#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_zoo_gpu.py tests/test_fused_gpu.py -m gpu > gpurun_out/t_pol2b.log 2>&1 || { tail -40 gpurun_out/t_pol2b.log; exit 1; }
tail -2 gpurun_out/t_pol2b.log
MODEL=inception_v3_slim_old STEPS=15 ROUNDS=5 VARIANTS="pol2=;pol1=pol2:0" timeout -k 10 300 python -u tools/ab_step.py > gpurun_out/r2_ab_policy2b_inception.log 2>&1 || { tail -20 gpurun_out/r2_ab_policy2b_inception.log; exit 1; }
tail -2 gpurun_out/r2_ab_policy2b_inception.log
timeout -k 10 300 python bench.py --model inception_v3_slim_old > gpurun_out/bench_inc_pol2.log 2>&1 || { tail -20 gpurun_out/bench_inc_pol2.log; exit 1; }
grep -o '"value": [0-9.]*, "unit": "images/sec", "n_gpus": [0-9]*, "steps": [0-9]*, "warmup": [0-9]*, "ms_per_step": [0-9.]*' gpurun_out/bench_inc_pol2.log
