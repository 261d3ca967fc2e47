#!/bin/bash
# Round 4: merged-head tile rule - numerics (merged vs per-head kernels, merged-forward model test, Inception DP
# gradients) and Inception-v3 same-process A/B (stile 1/0) + bench.
set -o pipefail
mkdir -p gpurun_out/r4
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_fused_ops_gpu.py -m gpu -k "merged_head_forward" > gpurun_out/r4/pytest_s20.log 2>&1
rc=$?; grep -E "PASSED|FAILED" gpurun_out/r4/pytest_s20.log | cut -c1-150; tail -1 gpurun_out/r4/pytest_s20.log
if [ $rc -ne 0 ]; then exit $rc; fi
MODEL=inception_v3_slim_old VARIANTS="base=;nostile=stile:0" STEPS=8 ROUNDS=6 timeout -k 10 400 python -u tools/ab_step.py > gpurun_out/r4/ab_stile_inception.log 2>&1 || { tail -30 gpurun_out/r4/ab_stile_inception.log; exit 1; }
tail -3 gpurun_out/r4/ab_stile_inception.log
timeout -k 10 240 python -u bench.py --model inception_v3_slim_old --steps 30 --warmup 5 > gpurun_out/r4/bench_inception_s20.log 2>&1 || { tail -30 gpurun_out/r4/bench_inception_s20.log; exit 1; }
tail -1 gpurun_out/r4/bench_inception_s20.log | cut -c1-200
