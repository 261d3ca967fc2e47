#!/bin/bash
# Round 5 session 39: Inception logits pool as the global mean, plain max-pool backward reading the concat-gradient slice in place - tests, same-box A/B (base = previous tree copy).
set -o pipefail
mkdir -p gpurun_out/r5
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_kernels_gpu.py tests/test_engine.py tests/test_trajectory_inception_gpu.py tests/test_zoo_gpu.py -m gpu -k "pool or inception or hipgraph or trajectory" > gpurun_out/r5/r5_s39_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/r5/r5_s39_pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/r5/r5_s39_pytest.log | head; exit $rc; }
for m in inception_v3_slim_old; do
  for v in base new base new; do
    if [ $v = base ]; then B=$R/ab_so/base_tree/bench.py; else B=$R/bench.py; fi
    timeout -k 10 200 python -u $B --model $m --steps 30 --warmup 5 > gpurun_out/r5/r5_s39_$m.$v.log 2>&1 || { echo "bench $m $v failed"; tail -5 gpurun_out/r5/r5_s39_$m.$v.log; exit 1; }
    echo "$m $v $(tail -1 gpurun_out/r5/r5_s39_$m.$v.log | grep -o '"value": [0-9.]*')"
  done
done
echo done
