#!/bin/bash
# Round 3, DP correctness on the GPU box: GPU suite, 8-rank shared-GPU gloo rehearsal of bench.py
# (the driver's N=8 launch shape; RCCL refuses several ranks per device), 1-GPU headline bench.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 420 python bench.py --gpus 8 --dist-backend gloo --batch 32 --steps 5 --warmup 2 > gpurun_out/bench_gloo8.log 2>&1 || { echo "gloo8 failed"; tail -30 gpurun_out/bench_gloo8.log; exit 1; }
grep '"value"' gpurun_out/bench_gloo8.log | cut -c1-600
timeout -k 10 300 python bench.py > gpurun_out/bench1.log 2>&1 || { tail -20 gpurun_out/bench1.log; exit 1; }
grep '"value"' gpurun_out/bench1.log | cut -c1-400
