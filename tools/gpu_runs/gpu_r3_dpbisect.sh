#!/bin/bash
# Bisect the 2-rank (gloo, shared GPU) BSP test against the round-3 knobs that are off by default.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in "DTM_SIBLING_GROUP=1 DTM_WGRAD_STREAM=0" "DTM_SIBLING_GROUP=1" "DTM_ACT_HANDOFF=1"; do
  env $v timeout -k 10 200 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_distributed.py -k "hip_kernels_match_single" > gpurun_out/dpbisect.log 2>&1
  rc=$?
  echo "$v -> rc=$rc $(tail -1 gpurun_out/dpbisect.log)"
  grep -E "Greatest|Mismatched" gpurun_out/dpbisect.log | head -3
  if [ $rc -ge 124 ]; then exit $rc; fi
done
