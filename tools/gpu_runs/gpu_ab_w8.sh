set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_fused_ops_gpu.py tests/test_fused_gpu.py -m gpu > gpurun_out/t_kern.log 2>&1 || { tail -40 gpurun_out/t_kern.log; exit 1; }
tail -1 gpurun_out/t_kern.log
VARIANTS="w8=;now8=w8:0" ROUNDS=5 timeout -k 10 400 python -u tools/ab_step.py > gpurun_out/ab_w8.log 2>&1 || { tail -20 gpurun_out/ab_w8.log; exit 1; }
tail -3 gpurun_out/ab_w8.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1 || { tail -20 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
STATS=1 TILES=-1,21,40 ROUNDS=3 timeout -k 10 600 python -u tools/conv_tile_sweep.py > gpurun_out/sweep_stats.log 2>&1 || { tail -30 gpurun_out/sweep_stats.log; exit 1; }
tail -1 gpurun_out/sweep_stats.log
