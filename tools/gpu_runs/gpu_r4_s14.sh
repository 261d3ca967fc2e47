#!/bin/bash
# Round 4: the split store as a compile-time epilogue variant (working tree) vs the runtime branch (86fee36) vs
# 983745b (before the split epilogue): ResNet-50 bench alternated 3x on one box; then the merged-forward tests
# (the split variant's numerics) and Inception bench.
set -o pipefail
mkdir -p gpurun_out/r4
export TMPDIR=/tmp
ROOT=$(pwd)
for i in 1 2 3; do
  for c in 983745b 86fee36 HEAD; do
    d=$ROOT; [ $c != HEAD ] && d=$ROOT/_bisect/$c
    (cd $d && timeout -k 10 200 python -u bench.py --steps 30 --warmup 5 > $ROOT/gpurun_out/r4/bench_fix_${c}_$i.log 2>&1)
    rc=$?
    echo "commit $c run $i rc=$rc: $(tail -1 gpurun_out/r4/bench_fix_${c}_$i.log | cut -c100-160)"
    if [ $rc -ne 0 ]; then exit $rc; fi
  done
done
timeout -k 10 400 python -u -m pytest -v -s --timeout 300 --timeout-method thread tests/test_kernels_gpu.py tests/test_fused_ops_gpu.py -m gpu -k "multi or merged or sibling" > gpurun_out/r4/pytest_split_variant.log 2>&1
rc=$?
grep -E "PASSED|FAILED" gpurun_out/r4/pytest_split_variant.log | cut -c1-150; tail -1 gpurun_out/r4/pytest_split_variant.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 240 python -u bench.py --model inception_v3_slim_old --steps 30 --warmup 5 > gpurun_out/r4/bench_inception_s14.log 2>&1 || { tail -30 gpurun_out/r4/bench_inception_s14.log; exit 1; }
tail -1 gpurun_out/r4/bench_inception_s14.log | cut -c1-200
