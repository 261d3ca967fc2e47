#!/bin/bash
# Round 5 session 38: 17x17 1x7 / 7x1 and 8x8 1x3 / 3x1 wgrad tile rules - tests, A/B benches.
set -o pipefail
mkdir -p gpurun_out/r5
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_fused_ops_gpu.py -m gpu -k "wgrad or sibling or multi" > gpurun_out/r5/r5_s38_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/r5/r5_s38_pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/r5/r5_s38_pytest.log | head; exit $rc; }
for m in inception_v3_slim_old; do
  for v in base new base new; do
    if [ $v = base ]; then export DTM_KERNELS_SO=$R/ab_so/libdtm_kernels_base.so; else unset DTM_KERNELS_SO; fi
    timeout -k 10 200 python -u bench.py --model $m --steps 30 --warmup 5 > gpurun_out/r5/r5_s38_$m.$v.log 2>&1 || { echo "bench $m $v failed"; tail -5 gpurun_out/r5/r5_s38_$m.$v.log; exit 1; }
    echo "$m $v $(tail -1 gpurun_out/r5/r5_s38_$m.$v.log | grep -o '"value": [0-9.]*')"
  done
done
echo done
