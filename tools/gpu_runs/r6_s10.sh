#!/bin/bash
# Round 6 session 10: stem wgrad with the BN backward fused on the pipelined 64x256 tile (14/15/16): numerics vs the
# unfused path, tile sweep.
set -o pipefail
mkdir -p gpurun_out/r6
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -m gpu -k "stem_wgrad_bn_fused" > gpurun_out/r6/r6_s10_pytest.log 2>&1 || { tail -30 gpurun_out/r6/r6_s10_pytest.log; exit 1; }
tail -1 gpurun_out/r6/r6_s10_pytest.log
TILES=-1 WTILES="-1,7,14,15,16,15:2,16:2,11" ROUNDS=5 timeout -k 10 300 python -u tools/stem_sweep.py > gpurun_out/r6/r6_s10_stem_wgrad.log 2>&1 || { tail -20 gpurun_out/r6/r6_s10_stem_wgrad.log; exit 1; }
cat gpurun_out/r6/r6_s10_stem_wgrad.log
