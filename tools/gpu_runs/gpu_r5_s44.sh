#!/bin/bash
# Round 5 session 44: XCD-aware block order in the grid-stride pool kernels (3x3/1 avg strips, 3x3/2 max pairs) -
# pool microbench base vs new .so, tests, same-box A/B vs HEAD tree (Inception + ResNet-50).
set -o pipefail
mkdir -p gpurun_out/r5
R=$GRAFT_REPO_ROOT
for v in base new; do
  if [ $v = base ]; then export DTM_KERNELS_SO=$R/ab_so/libdtm_kernels_base.so; else unset DTM_KERNELS_SO; fi
  timeout -k 10 120 python -u tools/pool_bench.py > gpurun_out/r5/r5_s44_poolbench_max.$v.log 2>&1 || { echo "poolbench $v failed"; tail -5 gpurun_out/r5/r5_s44_poolbench_max.$v.log; exit 1; }
  AVG=1 timeout -k 10 120 python -u tools/pool_bench.py > gpurun_out/r5/r5_s44_poolbench_avg.$v.log 2>&1 || { echo "poolbench avg $v failed"; tail -5 gpurun_out/r5/r5_s44_poolbench_avg.$v.log; exit 1; }
  echo "== $v"; cat gpurun_out/r5/r5_s44_poolbench_max.$v.log gpurun_out/r5/r5_s44_poolbench_avg.$v.log
done
unset DTM_KERNELS_SO
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_zoo_gpu.py -m gpu -k "pool" > gpurun_out/r5/r5_s44_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/r5/r5_s44_pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/r5/r5_s44_pytest.log | head; exit $rc; }
for m in inception_v3_slim_old resnet_v1_50; do
  for v in base new base new; do
    if [ $v = base ]; then B=$R/ab_so/base_tree/bench.py; else B=$R/bench.py; fi
    timeout -k 10 200 python -u $B --model $m --steps 30 --warmup 5 > gpurun_out/r5/r5_s44_$m.$v.log 2>&1 || { echo "bench $m $v failed"; tail -5 gpurun_out/r5/r5_s44_$m.$v.log; exit 1; }
    echo "$m $v $(tail -1 gpurun_out/r5/r5_s44_$m.$v.log | grep -o '"value": [0-9.]*')"
  done
done
echo done
