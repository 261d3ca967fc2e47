#!/bin/bash
# Round 5 session 45 (late-round validation): the whole GPU suite, the four benches, a ResNet-50 kernel-stats profile + timeline, smoke.
set -o pipefail
mkdir -p gpurun_out/r5
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 700 python -u -m pytest -v --timeout 400 --timeout-method thread tests -m gpu > gpurun_out/r5/r5_s45_pytest_gpu.log 2>&1
rc=$?; echo "gpu suite rc=$rc"; grep -E "FAILED|ERROR" gpurun_out/r5/r5_s45_pytest_gpu.log | head -10; tail -1 gpurun_out/r5/r5_s45_pytest_gpu.log
case $rc in 0|1) ;; *) exit $rc ;; esac
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5/r5_s45_smoke.log 2>&1; tail -1 gpurun_out/r5/r5_s45_smoke.log
for m in resnet_v1_50 inception_v3_slim_old vgg_16 lenet; do
  timeout -k 10 200 python -u bench.py --model $m --steps 20 --warmup 5 > gpurun_out/r5/r5_s45_bench_$m.log 2>&1 || { echo "bench $m failed"; tail -5 gpurun_out/r5/r5_s45_bench_$m.log; exit 1; }
  tail -1 gpurun_out/r5/r5_s45_bench_$m.log | cut -c1-160
done
rm -rf gpurun_out/r5/prof_s45
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r5/prof_s45 -o run --output-format csv -- python3 $R/bench.py --steps 8 --warmup 3 > $R/gpurun_out/r5/prof_s45.log 2>&1 || { echo "prof failed"; exit 1; }
cd $R
f=$(find gpurun_out/r5/prof_s45 -name "*kernel_stats.csv" | head -1); cp "$f" gpurun_out/r5/r5_s45_resnet50_kernel_stats.csv
t=$(find gpurun_out/r5/prof_s45 -name "*kernel_trace.csv" | head -1); python3 tools/step_timeline.py "$t" > gpurun_out/r5/r5_s45_timeline_resnet.txt; tail -1 gpurun_out/r5/r5_s45_timeline_resnet.txt
rm -rf gpurun_out/r5/prof_s45
echo done
# Inception-v3 captured-step kernel stats + timeline
rm -rf gpurun_out/r5/prof_s45i
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r5/prof_s45i -o run --output-format csv -- python3 $R/bench.py --model inception_v3_slim_old --steps 4 --warmup 3 > $R/gpurun_out/r5/prof_s45i.log 2>&1 || { echo "prof inception failed"; exit 1; }
cd $R
f=$(find gpurun_out/r5/prof_s45i -name "*kernel_stats.csv" | head -1); cp "$f" gpurun_out/r5/r5_s45_inception_kernel_stats.csv
t=$(find gpurun_out/r5/prof_s45i -name "*kernel_trace.csv" | head -1); python3 tools/step_timeline.py "$t" > gpurun_out/r5/r5_s45_timeline_inception.txt; tail -1 gpurun_out/r5/r5_s45_timeline_inception.txt
rm -rf gpurun_out/r5/prof_s45i
timeout -k 10 200 python -u bench.py --model inception_v3_slim_old --graph 0 --steps 20 --warmup 5 > gpurun_out/r5/r5_s45_bench_inception_eager.log 2>&1 || { echo "eager bench failed"; exit 1; }
tail -1 gpurun_out/r5/r5_s45_bench_inception_eager.log | cut -c1-160
echo done2
