#!/bin/bash
# ResNet-50 step timeline (kernel trace, both streams) with the side-stream weight gradients.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/prof_tl
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_tl -o run -- python3 bench.py --steps 3 --warmup 2 > gpurun_out/prof_tl.log 2>&1 || { echo "prof failed"; tail -30 gpurun_out/prof_tl.log; exit 1; }
f=$(find gpurun_out/prof_tl -name "*kernel_trace.csv" | head -1)
python3 tools/step_timeline.py "$f" > gpurun_out/r3_timeline_side.txt
tail -1 gpurun_out/r3_timeline_side.txt
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_fused_ops_gpu.py -k "side or stem" > gpurun_out/tl_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/tl_tests.log; exit 1; }
tail -1 gpurun_out/tl_tests.log
