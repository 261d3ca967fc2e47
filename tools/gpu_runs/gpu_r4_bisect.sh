#!/bin/bash
# Round 4: which commit fixed the round-3 sibling-merge DP mismatch (r3-style 2-rank, 2-step test with the merge on),
# then Inception-v3 same-process A/B of the merge + hand-off (now default on).
set -o pipefail
mkdir -p gpurun_out/r4
export TMPDIR=/tmp
ROOT=$(pwd)
for c in b42fb82 2c2a1ef 238e90f; do
  (cd _bisect/$c && DTM_SIBLING_GROUP=1 timeout -k 10 240 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_distributed.py -k "two_ranks_hip_kernels" > $ROOT/gpurun_out/r4/bisect_$c.log 2>&1)
  rc=$?
  echo "commit $c sibling=1: rc=$rc $(tail -1 gpurun_out/r4/bisect_$c.log | cut -c1-120)"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
MODEL=inception_v3_slim_old VARIANTS="base=;nosib=sib:0,ahand:0" STEPS=6 ROUNDS=5 timeout -k 10 400 python -u tools/ab_step.py > gpurun_out/r4/ab_sibling_inception.log 2>&1 || { tail -30 gpurun_out/r4/ab_sibling_inception.log; exit 1; }
tail -2 gpurun_out/r4/ab_sibling_inception.log
timeout -k 10 300 python -u bench.py --model inception_v3_slim_old --steps 20 --warmup 5 > gpurun_out/r4/bench_inception.log 2>&1 || { tail -30 gpurun_out/r4/bench_inception.log; exit 1; }
tail -1 gpurun_out/r4/bench_inception.log | cut -c1-200
