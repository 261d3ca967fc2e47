#!/bin/bash
# Round 6 session 17: occupancy variants of the register-staged block-output dgrads (epilogue row group 2, forced 4
# waves/SIMD): numerics, per-shape A/B, step A/B.
set -o pipefail
mkdir -p gpurun_out/r6
for v in 2 3; do
  DTM_ACT_OCC=$v timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -m gpu -k "act_dgrad_tiles" > gpurun_out/r6/r6_s17_pytest_$v.log 2>&1 || { tail -30 gpurun_out/r6/r6_s17_pytest_$v.log; exit 1; }
  tail -1 gpurun_out/r6/r6_s17_pytest_$v.log
done
TILES=4,3 KNOB=dtm_conv_set_act_occ VALUES=0,1,2,3 ROUNDS=5 timeout -k 10 300 python -u tools/act_dgrad_bench.py > gpurun_out/r6/r6_s17_act_occ.log 2>&1 || { tail -20 gpurun_out/r6/r6_s17_act_occ.log; exit 1; }
cat gpurun_out/r6/r6_s17_act_occ.log
VARIANTS="base=;o1=aocc:1;o2=aocc:2;o3=aocc:3;o2n2=aocc:2,nocc:2" ROUNDS=5 timeout -k 10 400 python -u tools/ab_step.py > gpurun_out/r6/r6_s17_ab_aocc.log 2>&1 || { tail -20 gpurun_out/r6/r6_s17_ab_aocc.log; exit 1; }
tail -4 gpurun_out/r6/r6_s17_ab_aocc.log
KNOB=dtm_conv_set_nt_occ VALUES=0,2,3 ONLY=56_256_64_1,28_512_128_1,56_64_256_1,28_256_128_1 PASSES=fwd,dgrad timeout -k 10 300 python -u tools/knob_ab.py > gpurun_out/r6/r6_s17_nt_occ.log 2>&1 || { tail -20 gpurun_out/r6/r6_s17_nt_occ.log; exit 1; }
cat gpurun_out/r6/r6_s17_nt_occ.log
