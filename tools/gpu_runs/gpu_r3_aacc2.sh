#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_fused_ops_gpu.py -k "direct3x3 or chain or full_window or block_output" > gpurun_out/aacc2_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/aacc2_tests.log; exit 1; }
tail -1 gpurun_out/aacc2_tests.log
MODEL=inception_v3_slim_old VARIANTS="direct=dir3:1;gemm=dir3:0" ROUNDS=6 timeout -k 10 400 python -u tools/ab_step.py > gpurun_out/dir3_inc5.log 2>&1 || { tail -30 gpurun_out/dir3_inc5.log; exit 1; }
tail -3 gpurun_out/dir3_inc5.log
VARIANTS="sact0=sact:0;sact1=sact:1" ROUNDS=5 timeout -k 10 400 python -u tools/ab_step.py > gpurun_out/sact_rn2.log 2>&1 || { tail -30 gpurun_out/sact_rn2.log; exit 1; }
tail -3 gpurun_out/sact_rn2.log
bash tools/gpu_runs/gpu_r3_inc.sh
grep "conv3x3_direct" gpurun_out/r3_timeline_inc.txt | cut -c1-110
