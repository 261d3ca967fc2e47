#!/bin/bash
# Round 6 session 35 (checkpoint after the direct 3x3 wgrad): whole GPU suite, smoke, the four benches +
# Inception eager + the no-flag default, and a kernel-stats profile of the ResNet-50 bench.
set -o pipefail
mkdir -p gpurun_out/r6
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/r6/r6_s35_pytest_gpu.log 2>&1
rc=$?; echo "gpu suite rc=$rc"; grep -E "FAILED|ERROR" gpurun_out/r6/r6_s35_pytest_gpu.log | head -10; tail -1 gpurun_out/r6/r6_s35_pytest_gpu.log
case $rc in 0|1) ;; *) exit $rc ;; esac
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6/r6_s35_smoke.log 2>&1; tail -1 gpurun_out/r6/r6_s35_smoke.log
for m in resnet_v1_50 inception_v3_slim_old vgg_16 lenet; do
  timeout -k 10 200 python -u bench.py --model $m --steps 20 --warmup 5 > gpurun_out/r6/r6_s35_bench_$m.log 2>&1 || { echo "bench $m failed"; tail -5 gpurun_out/r6/r6_s35_bench_$m.log; exit 1; }
  tail -1 gpurun_out/r6/r6_s35_bench_$m.log | cut -c1-160
done
timeout -k 10 200 python -u bench.py --model inception_v3_slim_old --graph 0 --steps 20 --warmup 5 > gpurun_out/r6/r6_s35_bench_inception_eager.log 2>&1 || { echo "eager bench failed"; exit 1; }
tail -1 gpurun_out/r6/r6_s35_bench_inception_eager.log | cut -c1-160
timeout -k 10 200 python -u bench.py > gpurun_out/r6/r6_s35_bench_default.log 2>&1 || { echo "default bench failed"; exit 1; }
tail -1 gpurun_out/r6/r6_s35_bench_default.log | cut -c1-200
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r6/prof35 -o run -- python3 $R/bench.py --steps 10 --warmup 3 > $R/gpurun_out/r6/r6_s35_prof_bench.log 2>&1 || { echo "profile failed"; tail -5 $R/gpurun_out/r6/r6_s35_prof_bench.log; exit 1; }
cd $R
f=$(find gpurun_out/r6/prof35 -name "*kernel_stats.csv" | head -1); cp "$f" gpurun_out/r6/r6_s35_resnet_kernel_stats.csv
find gpurun_out/r6/prof35 -name "*.csv" -delete
head -25 gpurun_out/r6/r6_s35_resnet_kernel_stats.csv | cut -c1-150
echo done
