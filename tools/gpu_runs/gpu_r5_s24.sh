#!/bin/bash
# Round 5 session 24: the 64x256 pipelined wgrad tile for K % 128 != 0 - tests, Inception shape sweep, A/B benches.
set -o pipefail
mkdir -p gpurun_out/r5
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -m gpu -k "wgrad" > gpurun_out/r5/r5_s24_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/r5/r5_s24_pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/r5/r5_s24_pytest.log | head; exit $rc; }
SET=inception B=128 WTILES=10:0,11:0 WONLY=1 ROUNDS=3 timeout -k 10 400 python -u tools/conv_tile_sweep.py > gpurun_out/r5/r5_s24_wgrad_k64_sweep.log 2>&1 || { echo sweep failed; tail -5 gpurun_out/r5/r5_s24_wgrad_k64_sweep.log; exit 1; }
grep -v amdgpu gpurun_out/r5/r5_s24_wgrad_k64_sweep.log | tail -30
for m in inception_v3_slim_old; do
  for v in base new base new; do
    if [ $v = base ]; then export DTM_KERNELS_SO=$R/ab_so/libdtm_kernels_base.so; else unset DTM_KERNELS_SO; fi
    timeout -k 10 200 python -u bench.py --model $m --steps 30 --warmup 5 > gpurun_out/r5/r5_s24_$m.$v.log 2>&1 || { echo "bench $m $v failed"; tail -5 gpurun_out/r5/r5_s24_$m.$v.log; exit 1; }
    echo "$m $v $(tail -1 gpurun_out/r5/r5_s24_$m.$v.log | grep -o '"value": [0-9.]*')"
  done
done
echo done
