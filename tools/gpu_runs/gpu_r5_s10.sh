#!/bin/bash
# Round 5 session 10: the one-rank RCCL pytest alone, with progress lines.
set -o pipefail
mkdir -p gpurun_out/r5
export TMPDIR=/tmp
timeout -k 10 150 python -u -m pytest -v -s --timeout 120 --timeout-method thread tests/test_distributed.py -m gpu -k "rccl or two_ranks_hip" 2>&1 | tee gpurun_out/r5/r5_s10_rccl_test.log | grep -v "amdgpu.ids"
