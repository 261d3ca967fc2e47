#!/bin/bash
# Round 5 session 47: ResNet-50 captured step with / without the weight-gradient side stream (DTM_DISABLE=wgrad_stream),
# alternating on one box (the round-3 A/B predates this round's kernels).
set -o pipefail
mkdir -p gpurun_out/r5
for v in on off on off on off; do
  if [ $v = off ]; then export DTM_DISABLE=wgrad_stream; else unset DTM_DISABLE; fi
  timeout -k 10 200 python -u bench.py --steps 30 --warmup 5 > gpurun_out/r5/r5_s47_resnet.$v.log 2>&1 || { echo "bench $v failed"; tail -5 gpurun_out/r5/r5_s47_resnet.$v.log; exit 1; }
  echo "resnet wgrad_stream=$v $(tail -1 gpurun_out/r5/r5_s47_resnet.$v.log | grep -o '"value": [0-9.]*')"
done
echo done
