#!/bin/bash
# Tests for the shared materialised activation / arena-backed BN statistics / pipelined 64x128 wgrad tile; stem wgrad
# split-K sizing A/B (ResNet-50); 64x128 wgrad tile A/B (ResNet-50, Inception-v3); Inception-v3 bench.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_fused_ops_gpu.py tests/test_fused_gpu.py tests/test_zoo_gpu.py tests/test_kernels_gpu.py > gpurun_out/swc_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/swc_tests.log; exit 1; }
tail -1 gpurun_out/swc_tests.log
VARIANTS="base=;swc150=swc:150;swc200=swc:200;swc300=swc:300" ROUNDS=8 timeout -k 10 500 python -u tools/ab_step.py > gpurun_out/r3_ab_stem_wgrad_cus.log 2>&1 || { tail -30 gpurun_out/r3_ab_stem_wgrad_cus.log; exit 1; }
tail -4 gpurun_out/r3_ab_stem_wgrad_cus.log
VARIANTS="base=;p1=wp64:1;p2=wp64:2" ROUNDS=6 timeout -k 10 500 python -u tools/ab_step.py > gpurun_out/r3_ab_wgrad_p64_resnet.log 2>&1 || { tail -30 gpurun_out/r3_ab_wgrad_p64_resnet.log; exit 1; }
tail -3 gpurun_out/r3_ab_wgrad_p64_resnet.log
MODEL=inception_v3_slim_old GRAPH=1 VARIANTS="base=;p1=wp64:1;p2=wp64:2" ROUNDS=6 timeout -k 10 500 python -u tools/ab_step.py > gpurun_out/r3_ab_wgrad_p64_inception.log 2>&1 || { tail -30 gpurun_out/r3_ab_wgrad_p64_inception.log; exit 1; }
tail -3 gpurun_out/r3_ab_wgrad_p64_inception.log
timeout -k 10 300 python bench.py --model inception_v3_slim_old > gpurun_out/r3_bench_inception.log 2>&1 || { tail -20 gpurun_out/r3_bench_inception.log; exit 1; }
tail -1 gpurun_out/r3_bench_inception.log
