#!/bin/bash
# Round 4: act-dgrad LDS tile numerics + sweep, tile decisions of one ResNet-50 step, 2-step DP checks of the sibling merge.
set -o pipefail
mkdir -p gpurun_out/r4
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "act_dgrad or pipelined_tiles" > gpurun_out/r4/pytest_actdgrad.log 2>&1 || { tail -30 gpurun_out/r4/pytest_actdgrad.log; exit 1; }
tail -2 gpurun_out/r4/pytest_actdgrad.log
DTM_TILE_LOG=1 timeout -k 10 200 python -u bench.py --steps 1 --warmup 1 > gpurun_out/r4/tilelog_resnet.out 2> gpurun_out/r4/tilelog_resnet.err || { tail -30 gpurun_out/r4/tilelog_resnet.err; exit 1; }
ACT=1 TILES=-1,4,21,26,0 ROUNDS=3 timeout -k 10 400 python -u tools/conv_tile_sweep.py > gpurun_out/r4/sweep_actdgrad.log 2>&1 || { tail -30 gpurun_out/r4/sweep_actdgrad.log; exit 1; }
grep -E "dgact|weighted" gpurun_out/r4/sweep_actdgrad.log
timeout -k 10 300 python -u tools/dp_grad_diag.py resnet_v1_50 DTM_SIBLING_GROUP=1 --steps 2 > gpurun_out/r4/diag_resnet_sib_2steps.log 2>&1 || { tail -30 gpurun_out/r4/diag_resnet_sib_2steps.log; exit 1; }
grep -E "RESULT|tensors differ" gpurun_out/r4/diag_resnet_sib_2steps.log
DTM_SIBLING_GROUP=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_distributed.py -k "two_ranks_hip_kernels" > gpurun_out/r4/pytest_dp_r3test_sib.log 2>&1
echo "r3-style 2-step DP test with sibling: rc=$?"
tail -5 gpurun_out/r4/pytest_dp_r3test_sib.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r4/bench_resnet_actl.log 2>&1 || { tail -30 gpurun_out/r4/bench_resnet_actl.log; exit 1; }
tail -1 gpurun_out/r4/bench_resnet_actl.log
