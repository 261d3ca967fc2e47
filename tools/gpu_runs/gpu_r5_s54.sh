#!/bin/bash
# Round 5 session 54 (end-of-round check of the final tree, after the FC-view change): the whole GPU suite, smoke, the four benches + Inception eager.
set -o pipefail
mkdir -p gpurun_out/r5
timeout -k 10 700 python -u -m pytest -v --timeout 400 --timeout-method thread tests -m gpu > gpurun_out/r5/r5_s54_pytest_gpu.log 2>&1
rc=$?; echo "gpu suite rc=$rc"; grep -E "FAILED|ERROR" gpurun_out/r5/r5_s54_pytest_gpu.log | head -10; tail -1 gpurun_out/r5/r5_s54_pytest_gpu.log
case $rc in 0|1) ;; *) exit $rc ;; esac
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5/r5_s54_smoke.log 2>&1; tail -1 gpurun_out/r5/r5_s54_smoke.log
for m in resnet_v1_50 inception_v3_slim_old vgg_16 lenet; do
  timeout -k 10 200 python -u bench.py --model $m --steps 20 --warmup 5 > gpurun_out/r5/r5_s54_bench_$m.log 2>&1 || { echo "bench $m failed"; tail -5 gpurun_out/r5/r5_s54_bench_$m.log; exit 1; }
  tail -1 gpurun_out/r5/r5_s54_bench_$m.log | cut -c1-160
done
timeout -k 10 200 python -u bench.py --model inception_v3_slim_old --graph 0 --steps 20 --warmup 5 > gpurun_out/r5/r5_s54_bench_inception_eager.log 2>&1 || { echo "eager bench failed"; exit 1; }
tail -1 gpurun_out/r5/r5_s54_bench_inception_eager.log | cut -c1-160
timeout -k 10 200 python -u bench.py > gpurun_out/r5/r5_s54_bench_default.log 2>&1 || { echo "default bench failed"; exit 1; }
tail -1 gpurun_out/r5/r5_s54_bench_default.log | cut -c1-200
echo done
