#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > gpurun_out/t_fin.log 2>&1 || { tail -40 gpurun_out/t_fin.log; exit 1; }
tail -2 gpurun_out/t_fin.log
VARIANTS="fin=;nofin=fin:0" timeout -k 10 300 python -u tools/ab_step.py > gpurun_out/r2_ab_fin_fuse.log 2>&1 || { tail -20 gpurun_out/r2_ab_fin_fuse.log; exit 1; }
tail -2 gpurun_out/r2_ab_fin_fuse.log
MODEL=inception_v3_slim_old STEPS=15 ROUNDS=4 VARIANTS="fin=;nofin=fin:0" timeout -k 10 300 python -u tools/ab_step.py > gpurun_out/r2_ab_fin_fuse_inception.log 2>&1 || { tail -20 gpurun_out/r2_ab_fin_fuse_inception.log; exit 1; }
tail -2 gpurun_out/r2_ab_fin_fuse_inception.log
timeout -k 10 300 python bench.py > gpurun_out/bench_fin.log 2>&1 || { tail -20 gpurun_out/bench_fin.log; exit 1; }
tail -1 gpurun_out/bench_fin.log | cut -c1-250
