#!/bin/bash
# Round 5 session 28: merged-head wgrads on the 256x256 tile - ResNet-50 projection-unit shape check, tests, A/B benches.
set -o pipefail
mkdir -p gpurun_out/r5
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
SET=custom B=256 SHAPES_CUSTOM="14,512,1280,1,1,2,SAME,1;14,512,1280,1,1,1,SAME,1;28,256,640,1,1,2,SAME,1" WTILES=10:0,12:0 WONLY=1 ROUNDS=3 timeout -k 10 300 python -u tools/conv_tile_sweep.py > gpurun_out/r5/r5_s28_wgrad_resnet_proj_sweep.log 2>&1 || { echo sweep failed; tail -5 gpurun_out/r5/r5_s28_wgrad_resnet_proj_sweep.log; exit 1; }
grep -v amdgpu gpurun_out/r5/r5_s28_wgrad_resnet_proj_sweep.log | tail -5
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_fused_ops_gpu.py -m gpu -k "wgrad or sibling or multi" > gpurun_out/r5/r5_s28_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/r5/r5_s28_pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/r5/r5_s28_pytest.log | head; exit $rc; }
for m in inception_v3_slim_old resnet_v1_50; do
  for v in base new base new; do
    if [ $v = base ]; then export DTM_KERNELS_SO=$R/ab_so/libdtm_kernels_base.so; else unset DTM_KERNELS_SO; fi
    timeout -k 10 200 python -u bench.py --model $m --steps 30 --warmup 5 > gpurun_out/r5/r5_s28_$m.$v.log 2>&1 || { echo "bench $m $v failed"; tail -5 gpurun_out/r5/r5_s28_$m.$v.log; exit 1; }
    echo "$m $v $(tail -1 gpurun_out/r5/r5_s28_$m.$v.log | grep -o '"value": [0-9.]*')"
  done
done
echo done
