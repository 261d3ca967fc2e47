#!/bin/bash
# Round 5 session 42: compile-time-tap 5x5/3 VALID avg pool, 8-channel global mean pool (fwd split rows, bwd 32-bit
# index), on top of s41 (fused loss, aux pool tail) - tests, same-box A/B vs HEAD tree (Inception + ResNet-50), timeline.
set -o pipefail
mkdir -p gpurun_out/r5
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_kernels_gpu.py tests/test_engine.py tests/test_trajectory_inception_gpu.py tests/test_trajectory_gpu.py tests/test_zoo_gpu.py -m gpu -k "pool or global or inception or hipgraph or trajectory or tail or xent or loss or resnet" > gpurun_out/r5/r5_s42_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/r5/r5_s42_pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/r5/r5_s42_pytest.log | head; exit $rc; }
for m in inception_v3_slim_old resnet_v1_50; do
  for v in base new base new; do
    if [ $v = base ]; then B=$R/ab_so/base_tree/bench.py; else B=$R/bench.py; fi
    timeout -k 10 200 python -u $B --model $m --steps 30 --warmup 5 > gpurun_out/r5/r5_s42_$m.$v.log 2>&1 || { echo "bench $m $v failed"; tail -5 gpurun_out/r5/r5_s42_$m.$v.log; exit 1; }
    echo "$m $v $(tail -1 gpurun_out/r5/r5_s42_$m.$v.log | grep -o '"value": [0-9.]*')"
  done
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r5/prof_s42i -o run --output-format csv -- python3 $R/bench.py --model inception_v3_slim_old --steps 4 --warmup 3 > $R/gpurun_out/r5/prof_s42i.log 2>&1 || { echo "prof inception failed"; exit 1; }
cd $R
f=$(find gpurun_out/r5/prof_s42i -name "*kernel_stats.csv" | head -1); cp "$f" gpurun_out/r5/r5_s42_inception_kernel_stats.csv
t=$(find gpurun_out/r5/prof_s42i -name "*kernel_trace.csv" | head -1); python3 tools/step_timeline.py "$t" > gpurun_out/r5/r5_s42_timeline_inception.txt; tail -1 gpurun_out/r5/r5_s42_timeline_inception.txt
rm -rf gpurun_out/r5/prof_s42i
echo done
