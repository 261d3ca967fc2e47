#!/bin/bash
# stride-decomposed dgrad: kernel tests, strided shapes of the conv table, whole-step A/B (ResNet-50, Inception-v3)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_dgrad_decomposition.py tests/test_kernels_gpu.py -m gpu > gpurun_out/dec_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/dec_tests.log; exit 1; }
tail -2 gpurun_out/dec_tests.log
ONLY=${ONLY:-_3} timeout -k 10 200 python -u tools/conv_microbench.py > gpurun_out/dec_table.txt 2>&1 || { tail -20 gpurun_out/dec_table.txt; exit 1; }
grep -v "^/opt" gpurun_out/dec_table.txt
VARIANTS="dec=;nodec=dec:0" timeout -k 10 300 python -u tools/ab_step.py > gpurun_out/r2_ab_dgrad_dec.log 2>&1 || { tail -20 gpurun_out/r2_ab_dgrad_dec.log; exit 1; }
tail -2 gpurun_out/r2_ab_dgrad_dec.log
MODEL=inception_v3_slim_old VARIANTS="dec=;nodec=dec:0" timeout -k 10 300 python -u tools/ab_step.py > gpurun_out/r2_ab_dgrad_dec_inception.log 2>&1 || { tail -20 gpurun_out/r2_ab_dgrad_dec_inception.log; exit 1; }
tail -2 gpurun_out/r2_ab_dgrad_dec_inception.log
