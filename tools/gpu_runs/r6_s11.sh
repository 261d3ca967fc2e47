#!/bin/bash
# Round 6 session 11: staggered w8 main loop (waves 4-7 defer each k-tile's second half past the next barrier):
# numerics, per-shape A/B on the layers the policy sends to w8, step A/B.
set -o pipefail
mkdir -p gpurun_out/r6
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -m gpu -k "(pipelined_tiles_match_reference or act_dgrad_tiles) and 40" > gpurun_out/r6/r6_s11_pytest.log 2>&1 || { tail -30 gpurun_out/r6/r6_s11_pytest.log; exit 1; }
tail -1 gpurun_out/r6/r6_s11_pytest.log
KNOB=dtm_conv_set_w8_stag VALUES=0,1 TILE=40 ONLY=14_,7_,28_256_512,28_128_512 timeout -k 10 300 python -u tools/knob_ab.py > gpurun_out/r6/r6_s11_stag.log 2>&1 || { tail -20 gpurun_out/r6/r6_s11_stag.log; exit 1; }
cat gpurun_out/r6/r6_s11_stag.log
VARIANTS="stag=;nostag=stag:0" ROUNDS=5 timeout -k 10 300 python -u tools/ab_step.py > gpurun_out/r6/r6_s11_ab_stag.log 2>&1 || { tail -20 gpurun_out/r6/r6_s11_ab_stag.log; exit 1; }
tail -2 gpurun_out/r6/r6_s11_ab_stag.log
