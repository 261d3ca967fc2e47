#!/bin/bash
# Round 4: weight gradients on the side stream inside the captured (hipGraph) step - numerics vs eager, then
# Inception-v3 bench A/B (DTM_GRAPH_SIDE 0/1, alternated twice).
set -o pipefail
mkdir -p gpurun_out/r4
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -v -s --timeout 300 --timeout-method thread tests/test_engine.py -m gpu -k "hipgraph or deterministic" > gpurun_out/r4/pytest_graphside.log 2>&1
rc=$?
# plain test failures (rc 1) still allow the benches; a crash, abort or time limit ends the call
if [ $rc -ne 0 ]; then grep -E "FAILED|Error|assert" gpurun_out/r4/pytest_graphside.log | head -30; fi
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
tail -8 gpurun_out/r4/pytest_graphside.log
for i in 1 2; do
  for gs in 0 1; do
    DTM_GRAPH_SIDE=$gs timeout -k 10 240 python -u bench.py --model inception_v3_slim_old --steps 30 --warmup 5 > gpurun_out/r4/bench_inception_gside${gs}_$i.log 2>&1 || { tail -30 gpurun_out/r4/bench_inception_gside${gs}_$i.log; exit 1; }
    echo "gside=$gs run $i: $(tail -1 gpurun_out/r4/bench_inception_gside${gs}_$i.log | cut -c1-170)"
  done
done
