#!/bin/bash
# Round 4 session start: smoke, ResNet-50 bench, step-1 DP gradient diagnostics (2 gloo ranks vs 1).
set -o pipefail
mkdir -p gpurun_out/r4
export TMPDIR=/tmp
timeout -k 10 300 python -u __graft_entry__.py smoke > gpurun_out/r4/smoke.log 2>&1 || { tail -30 gpurun_out/r4/smoke.log; exit 1; }
tail -1 gpurun_out/r4/smoke.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r4/bench_resnet.log 2>&1 || { tail -30 gpurun_out/r4/bench_resnet.log; exit 1; }
tail -1 gpurun_out/r4/bench_resnet.log
for spec in "resnet_v1_50" "resnet_v1_50 DTM_SIBLING_GROUP=1" "inception_v3_slim_old" "inception_v3_slim_old DTM_SIBLING_GROUP=1 DTM_ACT_HANDOFF=1" "vgg_16"; do
  tag=$(echo $spec | tr ' =' '__')
  timeout -k 10 300 python -u tools/dp_grad_diag.py $spec > gpurun_out/r4/diag_$tag.log 2>&1 || { echo "diag $spec rc=$?"; tail -30 gpurun_out/r4/diag_$tag.log; exit 1; }
  echo "== $spec"; grep -E "RESULT|tensors differ" gpurun_out/r4/diag_$tag.log
done
