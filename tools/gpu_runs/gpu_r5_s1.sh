#!/bin/bash
# Round 5 session 1: counters available, BN-sync GPU test (convex combine), ResNet-50 bench, Inception-v3
# eager (--graph 0) vs captured bench, HBM bytes per kernel (FETCH_SIZE / WRITE_SIZE passes).
set -o pipefail
mkdir -p gpurun_out/r5
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
(cd /tmp && timeout -k 10 60 rocprofv3 --list-avail > $R/gpurun_out/r5/avail.txt 2>&1) || echo "list-avail rc=$?"
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_distributed.py -m gpu -k "bn_moving or step1_gradients" > gpurun_out/r5/r5_s1_pytest_dp.log 2>&1 || { tail -40 gpurun_out/r5/r5_s1_pytest_dp.log; exit 1; }
tail -2 gpurun_out/r5/r5_s1_pytest_dp.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r5/r5_s1_bench_resnet.log 2>&1 || { tail -30 gpurun_out/r5/r5_s1_bench_resnet.log; exit 1; }
tail -1 gpurun_out/r5/r5_s1_bench_resnet.log | cut -c1-200
timeout -k 10 300 python -u bench.py --model inception_v3_slim_old --graph 1 --steps 20 --warmup 5 > gpurun_out/r5/r5_s1_bench_inception_graph.log 2>&1 || { tail -30 gpurun_out/r5/r5_s1_bench_inception_graph.log; exit 1; }
tail -1 gpurun_out/r5/r5_s1_bench_inception_graph.log | cut -c1-200
timeout -k 10 300 python -u bench.py --model inception_v3_slim_old --graph 0 --steps 20 --warmup 5 > gpurun_out/r5/r5_s1_bench_inception_eager.log 2>&1 || { tail -30 gpurun_out/r5/r5_s1_bench_inception_eager.log; exit 1; }
tail -1 gpurun_out/r5/r5_s1_bench_inception_eager.log | cut -c1-200
cd /tmp
timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/r5/pmc_fetch -o f -- python3 $R/bench.py --steps 4 --warmup 2 > $R/gpurun_out/r5/pmc_fetch.log 2>&1 || { echo "fetch pass failed"; tail -20 $R/gpurun_out/r5/pmc_fetch.log; exit 1; }
timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/r5/pmc_write -o w -- python3 $R/bench.py --steps 4 --warmup 2 > $R/gpurun_out/r5/pmc_write.log 2>&1 || { echo "write pass failed"; tail -20 $R/gpurun_out/r5/pmc_write.log; exit 1; }
cd $R
find gpurun_out/r5/pmc_fetch gpurun_out/r5/pmc_write -name "*.csv" | head
