#!/bin/bash
# Round 6 session 7: early side-input loads (conv_nt_kernel ESIDE) on the block-output dgrads: numerics, per-shape
# A/B, step A/B.
set -o pipefail
mkdir -p gpurun_out/r6
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_fused_ops_gpu.py -m gpu -k "act_dgrad_tiles or bnout or dgrad" > gpurun_out/r6/r6_s7_pytest.log 2>&1 || { tail -30 gpurun_out/r6/r6_s7_pytest.log; exit 1; }
tail -1 gpurun_out/r6/r6_s7_pytest.log
TILES=-1,4,3 ESIDE=0,1 ROUNDS=5 timeout -k 10 300 python -u tools/act_dgrad_bench.py > gpurun_out/r6/r6_s7_act_dgrad.log 2>&1 || { tail -20 gpurun_out/r6/r6_s7_act_dgrad.log; exit 1; }
cat gpurun_out/r6/r6_s7_act_dgrad.log
VARIANTS="eside=;noeside=eside:0" ROUNDS=5 timeout -k 10 300 python -u tools/ab_step.py > gpurun_out/r6/r6_s7_ab_eside.log 2>&1 || { tail -20 gpurun_out/r6/r6_s7_ab_eside.log; exit 1; }
tail -2 gpurun_out/r6/r6_s7_ab_eside.log
