#!/bin/bash
# Round 6 session 6: ADVICE r5 fixes on the GPU (aux pool tail with fused_bn off, deterministic bias sums,
# softmax-xent backward past grid.y), smoke with the loss-decrease check.
set -o pipefail
mkdir -p gpurun_out/r6
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_zoo_gpu.py tests/test_kernels_gpu.py -m gpu -k "aux_pool_tail or bias_column_sums or beyond_grid_y" > gpurun_out/r6/r6_s6_pytest.log 2>&1 || { tail -30 gpurun_out/r6/r6_s6_pytest.log; exit 1; }
tail -1 gpurun_out/r6/r6_s6_pytest.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6/r6_s6_smoke.log 2>&1 || { tail -10 gpurun_out/r6/r6_s6_smoke.log; exit 1; }
tail -1 gpurun_out/r6/r6_s6_smoke.log
