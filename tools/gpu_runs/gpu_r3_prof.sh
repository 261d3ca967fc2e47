#!/bin/bash
# Round 3 planning data: new GPU tests, ResNet-50 step timeline (kernel trace), aten call sites, Inception bench.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_trajectory_gpu.py tests/test_zoo_gpu.py -m gpu > gpurun_out/t_new.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/t_new.log; exit 1; }
tail -2 gpurun_out/t_new.log
timeout -k 10 300 python bench.py > gpurun_out/bench_rn.log 2>&1 || { tail -20 gpurun_out/bench_rn.log; exit 1; }
grep '"value"' gpurun_out/bench_rn.log | cut -c1-300
rm -rf gpurun_out/prof_rn
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_rn -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 2 > $GRAFT_REPO_ROOT/gpurun_out/prof_rn.log 2>&1 || { echo "prof failed"; tail -30 $GRAFT_REPO_ROOT/gpurun_out/prof_rn.log; exit 1; }
cd $GRAFT_REPO_ROOT
f=$(find gpurun_out/prof_rn -name "*kernel_trace.csv" | head -1)
python3 tools/step_timeline.py "$f" > gpurun_out/r3_timeline_resnet.txt
tail -1 gpurun_out/r3_timeline_resnet.txt
timeout -k 10 300 python tools/aten_sites.py --model resnet_v1_50 > gpurun_out/aten_resnet.txt 2>&1 || { echo "aten failed"; tail -20 gpurun_out/aten_resnet.txt; exit 1; }
head -30 gpurun_out/aten_resnet.txt
timeout -k 10 300 python bench.py --model inception_v3_slim_old > gpurun_out/bench_inc.log 2>&1 || { tail -20 gpurun_out/bench_inc.log; exit 1; }
grep '"value"' gpurun_out/bench_inc.log | cut -c1-300
timeout -k 10 120 ./tools/mfma_ab > gpurun_out/mfma_ab.log 2>&1 || { cat gpurun_out/mfma_ab.log; exit 1; }
cat gpurun_out/mfma_ab.log
