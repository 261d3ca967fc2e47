#!/bin/bash
# Round 4: hipGraph scratch-growth safety + CU-contention A/B (reserved CUs vs a comm-like co-resident kernel).
set -o pipefail
mkdir -p gpurun_out/r4
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_engine.py -m gpu -k "scratch or larger or graph" > gpurun_out/r4/pytest_graphsafe.log 2>&1
echo "graph-safety tests rc=$?"; tail -3 gpurun_out/r4/pytest_graphsafe.log
VARIANTS="base=;hog16=hog:16:8;hog16r=hog:16:8,rsv:16;hog32=hog:32:8;hog32r=hog:32:8,rsv:32" STEPS=6 ROUNDS=5 timeout -k 10 400 python -u tools/ab_step.py > gpurun_out/r4/ab_hog_reserve.log 2>&1 || { tail -30 gpurun_out/r4/ab_hog_reserve.log; exit 1; }
tail -6 gpurun_out/r4/ab_hog_reserve.log
