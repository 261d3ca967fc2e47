#!/bin/bash
# Round 4: merged sibling forward + grouped combine: numerics, same-process A/B (Inception-v3, ResNet-50), benches.
set -o pipefail
mkdir -p gpurun_out/r4
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_fused_ops_gpu.py -k "sibling" > gpurun_out/r4/pytest_sibling_s7.log 2>&1
echo "sibling tests rc=$?"; grep -E "PASS|FAIL|ERROR|assert" gpurun_out/r4/pytest_sibling_s7.log | cut -c1-200 | tail -12
MODEL=inception_v3_slim_old VARIANTS="base=;nofwd=sfwd:0;nocomb=scomb:0;neither=sfwd:0,scomb:0" STEPS=6 ROUNDS=5 timeout -k 10 500 python -u tools/ab_step.py > gpurun_out/r4/ab_sibfwd_inception.log 2>&1 || { tail -30 gpurun_out/r4/ab_sibfwd_inception.log; exit 1; }
tail -4 gpurun_out/r4/ab_sibfwd_inception.log
VARIANTS="base=;nofwd=sfwd:0" STEPS=6 ROUNDS=5 timeout -k 10 400 python -u tools/ab_step.py > gpurun_out/r4/ab_sibfwd_resnet.log 2>&1 || { tail -30 gpurun_out/r4/ab_sibfwd_resnet.log; exit 1; }
tail -2 gpurun_out/r4/ab_sibfwd_resnet.log
timeout -k 10 300 python -u bench.py --model inception_v3_slim_old --steps 20 --warmup 5 > gpurun_out/r4/bench_inception_s7.log 2>&1 || { tail -30 gpurun_out/r4/bench_inception_s7.log; exit 1; }
tail -1 gpurun_out/r4/bench_inception_s7.log | cut -c1-200
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r4/bench_resnet_s7.log 2>&1 || { tail -30 gpurun_out/r4/bench_resnet_s7.log; exit 1; }
tail -1 gpurun_out/r4/bench_resnet_s7.log | cut -c1-200
