#!/bin/bash
# Round 6 session 2: the ping-pong 256x256 tiles (conv_nt_pp_kernel = conv tile 41, conv_wgrad_pp_kernel = wgrad
# tile 13): numerics vs fp32, per-shape A/B against the w8 tiles (40 / 12), step-level A/B, default bench.
set -o pipefail
mkdir -p gpurun_out/r6
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -m gpu -k "((pipelined_tiles_match_reference or act_dgrad_tiles) and 41) or (wgrad_pipelined and (12 or 13))" > gpurun_out/r6/r6_s2_pytest_pp.log 2>&1 || { tail -30 gpurun_out/r6/r6_s2_pytest_pp.log; exit 1; }
tail -1 gpurun_out/r6/r6_s2_pytest_pp.log
TILES=40,41 STATS=1 ACT=1 ROUNDS=3 timeout -k 10 400 python -u tools/conv_tile_sweep.py > gpurun_out/r6/r6_s2_tiles_pp.log 2>&1 || { tail -20 gpurun_out/r6/r6_s2_tiles_pp.log; exit 1; }
tail -1 gpurun_out/r6/r6_s2_tiles_pp.log
WTILES=12,13 WONLY=1 ROUNDS=3 timeout -k 10 300 python -u tools/conv_tile_sweep.py > gpurun_out/r6/r6_s2_wtiles_pp.log 2>&1 || { tail -20 gpurun_out/r6/r6_s2_wtiles_pp.log; exit 1; }
tail -1 gpurun_out/r6/r6_s2_wtiles_pp.log
VARIANTS="pp=;w8=pp:0" ROUNDS=4 timeout -k 10 300 python -u tools/ab_step.py > gpurun_out/r6/r6_s2_ab_pp.log 2>&1 || { tail -20 gpurun_out/r6/r6_s2_ab_pp.log; exit 1; }
tail -2 gpurun_out/r6/r6_s2_ab_pp.log
timeout -k 10 200 python -u bench.py > gpurun_out/r6/r6_s2_bench_default.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/r6/r6_s2_bench_default.log; exit 1; }
tail -1 gpurun_out/r6/r6_s2_bench_default.log | cut -c1-200
