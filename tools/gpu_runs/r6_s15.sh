#!/bin/bash
# Round 6 session 15: RCCL collectives captured inside the hipGraph step (graph_comm) at world 1 vs eager.
set -o pipefail
mkdir -p gpurun_out/r6
timeout -k 10 240 python -u -m pytest -x -v -s --timeout 200 --timeout-method thread tests/test_distributed.py -m gpu -k "rccl" > gpurun_out/r6/r6_s15_pytest_rccl_graph.log 2>&1 || { tail -40 gpurun_out/r6/r6_s15_pytest_rccl_graph.log; exit 1; }
grep -E "PASS|FAIL|passed|failed" gpurun_out/r6/r6_s15_pytest_rccl_graph.log | tail -5
