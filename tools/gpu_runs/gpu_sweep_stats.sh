set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_fused_ops_gpu.py tests/test_fused_gpu.py -m gpu > gpurun_out/t_kern.log 2>&1 || { tail -40 gpurun_out/t_kern.log; exit 1; }
tail -2 gpurun_out/t_kern.log
STATS=1 TILES=${TILES:--1,0,4,21,40,43} ROUNDS=3 timeout -k 10 600 python -u tools/conv_tile_sweep.py > gpurun_out/sweep_stats.log 2>&1 || { tail -30 gpurun_out/sweep_stats.log; exit 1; }
grep -E "fwd |fwd\+s|dgrad|total" gpurun_out/sweep_stats.log
