#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > gpurun_out/t_defr.log 2>&1 || { tail -40 gpurun_out/t_defr.log; exit 1; }
tail -2 gpurun_out/t_defr.log
VARIANTS="defr=;imm=defr:0" timeout -k 10 300 python -u tools/ab_step.py > gpurun_out/r2_ab_def_reduce.log 2>&1 || { tail -20 gpurun_out/r2_ab_def_reduce.log; exit 1; }
tail -2 gpurun_out/r2_ab_def_reduce.log
MODEL=inception_v3_slim_old STEPS=15 ROUNDS=5 VARIANTS="defr=;imm=defr:0" timeout -k 10 300 python -u tools/ab_step.py > gpurun_out/r2_ab_def_reduce_inception.log 2>&1 || { tail -20 gpurun_out/r2_ab_def_reduce_inception.log; exit 1; }
tail -2 gpurun_out/r2_ab_def_reduce_inception.log
timeout -k 10 300 python bench.py --gpus 2 --dist-backend gloo --model lenet --steps 5 --warmup 3 > gpurun_out/bench_gloo2_defr.log 2>&1 || { tail -20 gpurun_out/bench_gloo2_defr.log; exit 1; }
grep -o '"value": [0-9.]*' gpurun_out/bench_gloo2_defr.log
