#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_fused_gpu.py -m gpu > gpurun_out/t_wn.log 2>&1 || { tail -40 gpurun_out/t_wn.log; exit 1; }
tail -2 gpurun_out/t_wn.log
VARIANTS="n256=;n128=wn256:0" timeout -k 10 300 python -u tools/ab_step.py > gpurun_out/r2_ab_wgrad_n256.log 2>&1 || { tail -20 gpurun_out/r2_ab_wgrad_n256.log; exit 1; }
tail -2 gpurun_out/r2_ab_wgrad_n256.log
