#!/bin/bash
# Round 5 session 17: the whole GPU suite, the four benches, a ResNet-50 kernel-stats profile + timeline, smoke.
set -o pipefail
mkdir -p gpurun_out/r5
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 700 python -u -m pytest -v --timeout 400 --timeout-method thread tests -m gpu > gpurun_out/r5/r5_s17_pytest_gpu.log 2>&1
rc=$?; echo "gpu suite rc=$rc"; grep -E "FAILED|ERROR" gpurun_out/r5/r5_s17_pytest_gpu.log | head -10; tail -1 gpurun_out/r5/r5_s17_pytest_gpu.log
case $rc in 0|1) ;; *) exit $rc ;; esac
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5/r5_s17_smoke.log 2>&1; tail -1 gpurun_out/r5/r5_s17_smoke.log
for m in resnet_v1_50 inception_v3_slim_old vgg_16 lenet; do
  timeout -k 10 200 python -u bench.py --model $m --steps 20 --warmup 5 > gpurun_out/r5/r5_s17_bench_$m.log 2>&1 || { echo "bench $m failed"; tail -5 gpurun_out/r5/r5_s17_bench_$m.log; exit 1; }
  tail -1 gpurun_out/r5/r5_s17_bench_$m.log | cut -c1-160
done
rm -rf gpurun_out/r5/prof_s17
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r5/prof_s17 -o run --output-format csv -- python3 $R/bench.py --steps 8 --warmup 3 > $R/gpurun_out/r5/prof_s17.log 2>&1 || { echo "prof failed"; exit 1; }
cd $R
f=$(find gpurun_out/r5/prof_s17 -name "*kernel_stats.csv" | head -1); cp "$f" gpurun_out/r5/r5_s17_resnet50_kernel_stats.csv
t=$(find gpurun_out/r5/prof_s17 -name "*kernel_trace.csv" | head -1); python3 tools/step_timeline.py "$t" > gpurun_out/r5/r5_s17_timeline_resnet.txt; tail -1 gpurun_out/r5/r5_s17_timeline_resnet.txt
rm -rf gpurun_out/r5/prof_s17
echo done
