#!/bin/bash
# Round 4: ResNet-50 bench at round-4 commits on ONE box (is there a regression across this round's changes?):
# 76af0c5 (round-4 start), 983745b (sibling merge on, before the merged forward), cf8af06 (merged forward +
# split epilogue), HEAD - alternated twice.  Then the Inception graph-vs-eager bit-exactness tests.
set -o pipefail
mkdir -p gpurun_out/r4
export TMPDIR=/tmp
ROOT=$(pwd)
for i in 1 2; do
  for c in 76af0c5 983745b cf8af06 HEAD; do
    d=$ROOT; [ $c != HEAD ] && d=$ROOT/_bisect/$c
    (cd $d && timeout -k 10 200 python -u bench.py --steps 30 --warmup 5 > $ROOT/gpurun_out/r4/bench_commit_${c}_$i.log 2>&1)
    rc=$?
    echo "commit $c run $i rc=$rc: $(tail -1 gpurun_out/r4/bench_commit_${c}_$i.log | cut -c100-190)"
    if [ $rc -ne 0 ]; then exit $rc; fi
  done
done
timeout -k 10 400 python -u -m pytest -v -s --timeout 300 --timeout-method thread tests/test_engine.py -m gpu -k "inception_bit_exact" > gpurun_out/r4/pytest_graph_inception_exact.log 2>&1
rc=$?
tail -4 gpurun_out/r4/pytest_graph_inception_exact.log
exit $rc
