#!/bin/bash
# Round 5 session 53: the loss reads an FC's padded output in place (row pitch) instead of a slice copy - tests,
# same-box A/B vs HEAD tree (Inception-v3, LeNet, VGG-16: 1001 / 10-class heads).
set -o pipefail
mkdir -p gpurun_out/r5
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_kernels_gpu.py tests/test_engine.py tests/test_zoo_gpu.py tests/test_trajectory_inception_gpu.py tests/test_trajectory_gpu.py tests/test_fused_ops_gpu.py -m gpu > gpurun_out/r5/r5_s53_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/r5/r5_s53_pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/r5/r5_s53_pytest.log | head; exit $rc; }
for m in inception_v3_slim_old lenet vgg_16; do
  for v in base new base new; do
    if [ $v = base ]; then B=$R/ab_so/base_tree/bench.py; else B=$R/bench.py; fi
    timeout -k 10 200 python -u $B --model $m --steps 30 --warmup 5 > gpurun_out/r5/r5_s53_$m.$v.log 2>&1 || { echo "bench $m $v failed"; tail -5 gpurun_out/r5/r5_s53_$m.$v.log; exit 1; }
    echo "$m $v $(tail -1 gpurun_out/r5/r5_s53_$m.$v.log | grep -o '"value": [0-9.]*')"
  done
done
echo done
