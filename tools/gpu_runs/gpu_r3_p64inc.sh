#!/bin/bash
# Merged backward of sibling 1x1 convs (Inception mixed blocks, ResNet projection units) + act-input hand-off:
# tests, eager A/Bs (+ pipelined 64x128 wgrad tile on Inception); ResNet-50 bench; Inception-v3 bench (one captured
# graph per process, the product path) last.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_fused_ops_gpu.py tests/test_fused_gpu.py tests/test_zoo_gpu.py > gpurun_out/sib_tests.log 2>&1 || { echo "tests failed"; grep -E "^E  |FAILED" gpurun_out/sib_tests.log | head -30; tail -2 gpurun_out/sib_tests.log; exit 1; }
tail -1 gpurun_out/sib_tests.log
VARIANTS="base=;sib=sib:1" ROUNDS=6 timeout -k 10 400 python -u tools/ab_step.py > gpurun_out/r3_ab_sibling_resnet.log 2>&1 || { tail -30 gpurun_out/r3_ab_sibling_resnet.log; exit 1; }
tail -2 gpurun_out/r3_ab_sibling_resnet.log
MODEL=inception_v3_slim_old VARIANTS="base=;sib=sib:1;ah=ahand:1;both=sib:1,ahand:1;p1=wp64:1" ROUNDS=6 timeout -k 10 500 python -u tools/ab_step.py > gpurun_out/r3_ab_sibling_p64_inception.log 2>&1 || { tail -30 gpurun_out/r3_ab_sibling_p64_inception.log; exit 1; }
tail -5 gpurun_out/r3_ab_sibling_p64_inception.log
timeout -k 10 300 python bench.py > gpurun_out/r3_bench_resnet.log 2>&1 || { tail -20 gpurun_out/r3_bench_resnet.log; exit 1; }
tail -1 gpurun_out/r3_bench_resnet.log
timeout -k 10 300 python bench.py --model inception_v3_slim_old > gpurun_out/r3_bench_inception.log 2>&1 || { tail -20 gpurun_out/r3_bench_inception.log; exit 1; }
tail -1 gpurun_out/r3_bench_inception.log
