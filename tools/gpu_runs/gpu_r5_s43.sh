#!/bin/bash
# Round 5 session 43: XCD-remapped 5x5/3 VALID avg pool kernels - tests, Inception timeline, same-box A/B vs HEAD tree.
set -o pipefail
mkdir -p gpurun_out/r5
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_zoo_gpu.py -m gpu -k "avgpool or tail or conv_tile or wgrad" > gpurun_out/r5/r5_s43_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/r5/r5_s43_pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/r5/r5_s43_pytest.log | head; exit $rc; }
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r5/prof_s43i -o run --output-format csv -- python3 $R/bench.py --model inception_v3_slim_old --steps 4 --warmup 3 > $R/gpurun_out/r5/prof_s43i.log 2>&1 || { echo "prof inception failed"; exit 1; }
cd $R
t=$(find gpurun_out/r5/prof_s43i -name "*kernel_trace.csv" | head -1); python3 tools/step_timeline.py "$t" > gpurun_out/r5/r5_s43_timeline_inception.txt; tail -1 gpurun_out/r5/r5_s43_timeline_inception.txt
grep -E "avgpool_(fwd|bwd)_valid" gpurun_out/r5/r5_s43_timeline_inception.txt
rm -rf gpurun_out/r5/prof_s43i
for m in inception_v3_slim_old; do
  for v in base new base new; do
    if [ $v = base ]; then B=$R/ab_so/base_tree/bench.py; else B=$R/bench.py; fi
    timeout -k 10 200 python -u $B --model $m --steps 30 --warmup 5 > gpurun_out/r5/r5_s43_$m.$v.log 2>&1 || { echo "bench $m $v failed"; tail -5 gpurun_out/r5/r5_s43_$m.$v.log; exit 1; }
    echo "$m $v $(tail -1 gpurun_out/r5/r5_s43_$m.$v.log | grep -o '"value": [0-9.]*')"
  done
done
echo done
