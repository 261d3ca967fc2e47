#!/bin/bash
# Round 4: sibling numerics (merged forward / grouped combine), the DP gradient matrix (1 vs 2 gloo ranks, configs
# looped per worker) + BN moving statistics across ranks, Inception merged-forward A/B, benches.
set -o pipefail
mkdir -p gpurun_out/r4
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_fused_ops_gpu.py -k "sibling" > gpurun_out/r4/pytest_sibling.log 2>&1
echo "sibling tests rc=$?"; grep -E "PASS|FAIL|ERROR" gpurun_out/r4/pytest_sibling.log | cut -c1-160 | tail -10
timeout -k 10 500 python -u -m pytest -v -s --timeout 450 --timeout-method thread tests/test_distributed.py -m gpu > gpurun_out/r4/pytest_dp_gpu.log 2>&1
echo "dp gpu tests rc=$?"; grep -E "PASS|FAIL|ERROR|assert" gpurun_out/r4/pytest_dp_gpu.log | cut -c1-300 | tail -12
MODEL=inception_v3_slim_old VARIANTS="base=;nofwd=sfwd:0" STEPS=6 ROUNDS=5 timeout -k 10 300 python -u tools/ab_step.py > gpurun_out/r4/ab_sibfwd_inception.log 2>&1 || { tail -30 gpurun_out/r4/ab_sibfwd_inception.log; exit 1; }
tail -2 gpurun_out/r4/ab_sibfwd_inception.log
timeout -k 10 200 python -u bench.py --model inception_v3_slim_old --steps 20 --warmup 5 > gpurun_out/r4/bench_inception_s7.log 2>&1 || { tail -30 gpurun_out/r4/bench_inception_s7.log; exit 1; }
tail -1 gpurun_out/r4/bench_inception_s7.log | cut -c1-200
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r4/bench_resnet_s7.log 2>&1 || { tail -30 gpurun_out/r4/bench_resnet_s7.log; exit 1; }
tail -1 gpurun_out/r4/bench_resnet_s7.log | cut -c1-200
