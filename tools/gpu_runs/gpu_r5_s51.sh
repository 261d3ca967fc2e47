#!/bin/bash
# Round 5 session 51: Inception-v3 with the weight-gradient side stream in the eager step (bench --graph 0
# --wgrad-stream 1) vs the eager single-stream step and the captured step (the default), alternating on one box.
set -o pipefail
mkdir -p gpurun_out/r5
for v in graph eager eside graph eager eside; do
  case $v in graph) A="";; eager) A="--graph 0";; eside) A="--graph 0 --wgrad-stream 1";; esac
  timeout -k 10 200 python -u bench.py --model inception_v3_slim_old --steps 30 --warmup 5 $A > gpurun_out/r5/r5_s51_inception.$v.log 2>&1 || { echo "bench $v failed"; tail -5 gpurun_out/r5/r5_s51_inception.$v.log; exit 1; }
  echo "inception $v $(tail -1 gpurun_out/r5/r5_s51_inception.$v.log | grep -o '"value": [0-9.]*')"
done
echo done
