#!/bin/bash
# correctness of every pipelined tile id, then the per-shape tile sweep ($TILES, $ONLY)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k pipelined -m gpu > gpurun_out/t_tiles.log 2>&1 || { tail -40 gpurun_out/t_tiles.log; exit 1; }
tail -2 gpurun_out/t_tiles.log
TILES=${TILES:--1,21,26,27,28,29} ROUNDS=3 timeout -k 10 600 python -u tools/conv_tile_sweep.py > gpurun_out/${OUT:-sweep.log} 2>&1 || { tail -30 gpurun_out/${OUT:-sweep.log}; exit 1; }
grep -v "^/opt" gpurun_out/${OUT:-sweep.log}
