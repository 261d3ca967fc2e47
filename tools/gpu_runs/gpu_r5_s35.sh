#!/bin/bash
# Round 5 session 35: bias column sums on the BN-statistics kernel, bf16 global average pool - tests, same-box A/B (base = previous tree copy).
set -o pipefail
mkdir -p gpurun_out/r5
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_engine.py tests/test_trajectory_gpu.py tests/test_zoo_gpu.py -m gpu -k "fc or xent or softmax or linear or hipgraph or trajectory or head or bias or global or resnet" > gpurun_out/r5/r5_s35_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/r5/r5_s35_pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/r5/r5_s35_pytest.log | head; exit $rc; }
for m in inception_v3_slim_old resnet_v1_50; do
  for v in base new base new; do
    if [ $v = base ]; then B=$R/ab_so/base_tree/bench.py; else B=$R/bench.py; fi
    timeout -k 10 200 python -u $B --model $m --steps 30 --warmup 5 > gpurun_out/r5/r5_s35_$m.$v.log 2>&1 || { echo "bench $m $v failed"; tail -5 gpurun_out/r5/r5_s35_$m.$v.log; exit 1; }
    echo "$m $v $(tail -1 gpurun_out/r5/r5_s35_$m.$v.log | grep -o '"value": [0-9.]*')"
  done
done
echo done
