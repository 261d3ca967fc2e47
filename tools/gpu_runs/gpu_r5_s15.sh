#!/bin/bash
# Round 5 session 15: BN-gradient sums of act / block-output dgrads by fp32 atomics (few pixel tiles) - kernel tests,
# the fused-op suite, same-box A/B benches against the previous build (ab_so/libdtm_kernels_base.so).
set -o pipefail
mkdir -p gpurun_out/r5
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py tests/test_dgrad_decomposition.py tests/test_fused_ops_gpu.py -m gpu > gpurun_out/r5/r5_s15_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/r5/r5_s15_pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/r5/r5_s15_pytest.log | head; exit $rc; }
for m in inception_v3_slim_old resnet_v1_50; do
  for v in base new base new; do
    if [ $v = base ]; then export DTM_KERNELS_SO=$R/ab_so/libdtm_kernels_base.so; else unset DTM_KERNELS_SO; fi
    timeout -k 10 200 python -u bench.py --model $m --steps 30 --warmup 5 > gpurun_out/r5/r5_s15_$m.$v.log 2>&1 || { echo "bench $m $v failed"; tail -5 gpurun_out/r5/r5_s15_$m.$v.log; exit 1; }
    echo "$m $v $(tail -1 gpurun_out/r5/r5_s15_$m.$v.log | grep -o '"value": [0-9.]*')"
  done
done
echo done
