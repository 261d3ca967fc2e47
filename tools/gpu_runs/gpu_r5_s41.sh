#!/bin/bash
# Round 5 session 41: fused training loss (mean xent heads + weights in one op), aux-head pool gradient added in place into the main-path gradient (pool_tail), 32-bit-index generic avg pool - tests, same-box A/B (base = previous tree copy).
set -o pipefail
mkdir -p gpurun_out/r5
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_kernels_gpu.py tests/test_engine.py tests/test_trajectory_inception_gpu.py tests/test_zoo_gpu.py -m gpu -k "pool or inception or hipgraph or trajectory or tail or xent or loss" > gpurun_out/r5/r5_s41_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/r5/r5_s41_pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/r5/r5_s41_pytest.log | head; exit $rc; }
for m in inception_v3_slim_old; do
  for v in base new notail base new notail; do
    if [ $v = base ]; then B=$R/ab_so/base_tree/bench.py; else B=$R/bench.py; fi
    if [ $v = notail ]; then export DTM_DISABLE=pool_tail; else unset DTM_DISABLE; fi; timeout -k 10 200 python -u $B --model $m --steps 30 --warmup 5 > gpurun_out/r5/r5_s41_$m.$v.log 2>&1 || { echo "bench $m $v failed"; tail -5 gpurun_out/r5/r5_s41_$m.$v.log; exit 1; }
    echo "$m $v $(tail -1 gpurun_out/r5/r5_s41_$m.$v.log | grep -o '"value": [0-9.]*')"
  done
done
echo done
# captured-step kernel stats + timeline of the new tree
export TMPDIR=/tmp
unset DTM_DISABLE
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r5/prof_s41i -o run --output-format csv -- python3 $R/bench.py --model inception_v3_slim_old --steps 4 --warmup 3 > $R/gpurun_out/r5/prof_s41i.log 2>&1 || { echo "prof inception failed"; exit 1; }
cd $R
f=$(find gpurun_out/r5/prof_s41i -name "*kernel_stats.csv" | head -1); cp "$f" gpurun_out/r5/r5_s41_inception_kernel_stats.csv
t=$(find gpurun_out/r5/prof_s41i -name "*kernel_trace.csv" | head -1); python3 tools/step_timeline.py "$t" > gpurun_out/r5/r5_s41_timeline_inception.txt; tail -1 gpurun_out/r5/r5_s41_timeline_inception.txt
rm -rf gpurun_out/r5/prof_s41i
echo done2
