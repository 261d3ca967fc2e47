#!/bin/bash
# Round 5 session 27: wgrad tiles on Inception-v3's merged sibling-head widths; A/B of the 64x256 tile rules.
set -o pipefail
mkdir -p gpurun_out/r5
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
SET=custom B=128 SHAPES_CUSTOM="17,768,704,1,1,1,SAME,2;17,768,768,1,1,1,SAME,1;17,768,640,1,1,1,SAME,1;17,768,384,1,1,1,SAME,1;35,288,240,1,1,1,SAME,1;35,256,240,1,1,1,SAME,1;35,192,208,1,1,1,SAME,1;8,2048,1344,1,1,1,SAME,1;8,1280,1344,1,1,1,SAME,1;35,288,64,1,1,1,SAME,1" WTILES=1:0,10:0,11:0,12:0 WONLY=1 ROUNDS=3 timeout -k 10 300 python -u tools/conv_tile_sweep.py > gpurun_out/r5/r5_s27_wgrad_heads_sweep.log 2>&1 || { echo sweep failed; tail -5 gpurun_out/r5/r5_s27_wgrad_heads_sweep.log; exit 1; }
grep -v amdgpu gpurun_out/r5/r5_s27_wgrad_heads_sweep.log | tail -14
for m in inception_v3_slim_old; do
  for v in base new base new; do
    if [ $v = base ]; then export DTM_KERNELS_SO=$R/ab_so/libdtm_kernels_base.so; else unset DTM_KERNELS_SO; fi
    timeout -k 10 200 python -u bench.py --model $m --steps 30 --warmup 5 > gpurun_out/r5/r5_s27_$m.$v.log 2>&1 || { echo "bench $m $v failed"; tail -5 gpurun_out/r5/r5_s27_$m.$v.log; exit 1; }
    echo "$m $v $(tail -1 gpurun_out/r5/r5_s27_$m.$v.log | grep -o '"value": [0-9.]*')"
  done
done
echo done
