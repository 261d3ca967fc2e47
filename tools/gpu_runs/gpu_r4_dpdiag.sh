#!/bin/bash
# Round 4: step-1 per-parameter DP gradient diagnostics (2 gloo ranks on the one GPU vs 1 rank) + graph-safety tests.
set -o pipefail
mkdir -p gpurun_out/r4
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/dp_grad_diag.py resnet_v1_50 DTM_SIBLING_GROUP=1 > gpurun_out/r4/diag_resnet_sib.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/dp_grad_diag.py resnet_v1_50 DTM_SIBLING_GROUP=1 --no-overlap > gpurun_out/r4/diag_resnet_sib_noov.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/dp_grad_diag.py resnet_v1_50 > gpurun_out/r4/diag_resnet_def.log 2>&1 || exit $?
timeout -k 10 300 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_engine.py -k "scratch_growth or larger_eager" > gpurun_out/r4/pytest_graphsafe.log 2>&1
echo "graphsafe rc=$?"
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_distributed.py -k "step1_gradients" > gpurun_out/r4/pytest_dp_matrix.log 2>&1
echo "pytest rc=$?"
tail -3 gpurun_out/r4/pytest_dp_matrix.log
grep -h RESULT gpurun_out/r4/diag_*.log
