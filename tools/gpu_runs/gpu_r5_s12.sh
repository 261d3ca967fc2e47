#!/bin/bash
# Round 5 session 12: latency-shaped reductions - kernel + DP tests, then same-box A/B benches (baseline .so = HEAD).
set -o pipefail
mkdir -p gpurun_out/r5
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py tests/test_distributed.py -m gpu > gpurun_out/r5/r5_s12_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r5/r5_s12_pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/r5/r5_s12_pytest.log | head; exit $rc; }
for m in resnet_v1_50 inception_v3_slim_old; do
  for v in base new base new; do
    if [ $v = base ]; then export DTM_KERNELS_SO=$R/ab_so/libdtm_kernels_base.so; else unset DTM_KERNELS_SO; fi
    timeout -k 10 200 python -u bench.py --model $m --steps 30 --warmup 5 > gpurun_out/r5/r5_s12_$m.$v.log 2>&1 || { echo "bench $m $v failed"; tail -5 gpurun_out/r5/r5_s12_$m.$v.log; exit 1; }
    echo "$m $v $(tail -1 gpurun_out/r5/r5_s12_$m.$v.log | cut -c1-120)"
  done
done
unset DTM_KERNELS_SO
echo done
