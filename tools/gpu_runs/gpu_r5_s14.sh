#!/bin/bash
# Round 5 session 14: widened register-staged wgrad column tiles (64x192 / 64x256) - tests, per-shape sweep with the
# BN-apply prologue, same-box A/B benches against the previous build (ab_so/libdtm_kernels_base.so).
set -o pipefail
mkdir -p gpurun_out/r5
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
#timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -m gpu -k "wgrad" > gpurun_out/r5/r5_s14_pytest.log 2>&1
#rc=$?; tail -2 gpurun_out/r5/r5_s14_pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/r5/r5_s14_pytest.log | head; exit $rc; }
#WTILES=1:0,7:0,9:0,8:0 WPRO=1 WONLY=1 ROUNDS=3 timeout -k 10 300 python -u tools/conv_tile_sweep.py > gpurun_out/r5/r5_s14_wgrad_wide_sweep.log 2>&1 || { echo sweep failed; tail -5 gpurun_out/r5/r5_s14_wgrad_wide_sweep.log; exit 1; }
#tail -2 gpurun_out/r5/r5_s14_wgrad_wide_sweep.log
for m in resnet_v1_50; do
  for v in base new base new; do
    if [ $v = base ]; then export DTM_KERNELS_SO=$R/ab_so/libdtm_kernels_base.so; else unset DTM_KERNELS_SO; fi
    timeout -k 10 200 python -u bench.py --model $m --steps 30 --warmup 5 > gpurun_out/r5/r5_s14b_$m.$v.log 2>&1 || { echo "bench $m $v failed"; tail -5 gpurun_out/r5/r5_s14b_$m.$v.log; exit 1; }
    echo "$m $v $(tail -1 gpurun_out/r5/r5_s14b_$m.$v.log | grep -o '"value": [0-9.]*')"
  done
done
echo done
