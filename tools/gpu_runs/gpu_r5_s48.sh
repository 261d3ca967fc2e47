#!/bin/bash
# Round 5 session 48: ResNet-50 step captured WITH the weight-gradient side stream (bench --graph 1 --graph-side 1) vs
# the eager side-stream step (the default) and the single-stream capture; the bit-exactness test first.
set -o pipefail
mkdir -p gpurun_out/r5
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_engine.py -m gpu -k "hipgraph" > gpurun_out/r5/r5_s48_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/r5/r5_s48_pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/r5/r5_s48_pytest.log | head; exit $rc; }
for v in eager gside g1 eager gside g1; do
  case $v in eager) A="";; gside) A="--graph 1 --graph-side 1";; g1) A="--graph 1";; esac
  timeout -k 10 200 python -u bench.py --steps 30 --warmup 5 $A > gpurun_out/r5/r5_s48_resnet.$v.log 2>&1 || { echo "bench $v failed"; tail -5 gpurun_out/r5/r5_s48_resnet.$v.log; exit 1; }
  echo "resnet $v $(tail -1 gpurun_out/r5/r5_s48_resnet.$v.log | grep -o '"value": [0-9.]*')"
done
echo done
