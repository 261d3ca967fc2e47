#!/bin/bash
# Round 5 session 30: stream-K 256x256 conv tile - tests, ResNet-50 shape sweep, same-box A/B benches.
set -o pipefail
mkdir -p gpurun_out/r5
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -m gpu -k "stream_k or conv" > gpurun_out/r5/r5_s30_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/r5/r5_s30_pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/r5/r5_s30_pytest.log | head; exit $rc; }
for v in base new; do
  if [ $v = base ]; then export DTM_KERNELS_SO=$R/ab_so/libdtm_kernels_base.so; else unset DTM_KERNELS_SO; fi
  SET=custom B=256 STATS=1 ROUNDS=3 TILES=-1 SHAPES_CUSTOM="14,256,256,3,3,1,SAME,6;14,1024,256,1,1,1,SAME,6;7,512,512,3,3,1,SAME,3;7,2048,512,1,1,1,SAME,3;14,512,1024,1,1,1,SAME,1" timeout -k 10 300 python -u tools/conv_tile_sweep.py > gpurun_out/r5/r5_s30_sweep.$v.log 2>&1 || { echo "sweep $v failed"; tail -5 gpurun_out/r5/r5_s30_sweep.$v.log; exit 1; }
  echo "== $v"; grep -v amdgpu gpurun_out/r5/r5_s30_sweep.$v.log | tail -26
done
unset DTM_KERNELS_SO
for m in resnet_v1_50; do
  for v in base new base new; do
    if [ $v = base ]; then export DTM_KERNELS_SO=$R/ab_so/libdtm_kernels_base.so; else unset DTM_KERNELS_SO; fi
    timeout -k 10 200 python -u bench.py --model $m --steps 30 --warmup 5 > gpurun_out/r5/r5_s30_$m.$v.log 2>&1 || { echo "bench $m $v failed"; tail -5 gpurun_out/r5/r5_s30_$m.$v.log; exit 1; }
    echo "$m $v $(tail -1 gpurun_out/r5/r5_s30_$m.$v.log | grep -o '"value": [0-9.]*')"
  done
done
echo done
