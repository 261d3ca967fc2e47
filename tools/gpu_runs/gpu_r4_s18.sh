#!/bin/bash
# Round 4: ResNet-50 with its merged forward opt-in (default off): merged-forward + DP gradient tests, bench x2.
set -o pipefail
mkdir -p gpurun_out/r4
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_fused_ops_gpu.py tests/test_distributed.py -m gpu -k "merged_head_forward or step1_gradients or merged_backward" > gpurun_out/r4/pytest_s18.log 2>&1
rc=$?; grep -E "PASSED|FAILED" gpurun_out/r4/pytest_s18.log | cut -c1-150; tail -1 gpurun_out/r4/pytest_s18.log
if [ $rc -ne 0 ]; then exit $rc; fi
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --steps 30 --warmup 5 > gpurun_out/r4/bench_resnet_s18_$i.log 2>&1 || { tail -20 gpurun_out/r4/bench_resnet_s18_$i.log; exit 1; }
  tail -1 gpurun_out/r4/bench_resnet_s18_$i.log | cut -c1-200
done
