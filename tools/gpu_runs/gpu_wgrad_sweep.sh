set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -m gpu -k "wgrad" > gpurun_out/t_kern.log 2>&1 || { tail -40 gpurun_out/t_kern.log; exit 1; }
tail -1 gpurun_out/t_kern.log
WONLY=1 WTILES=${WTILES:--1,12:1,12:2,12:3} ROUNDS=3 timeout -k 10 600 python -u tools/conv_tile_sweep.py > gpurun_out/sweep_wgrad.log 2>&1 || { tail -30 gpurun_out/sweep_wgrad.log; exit 1; }
cat gpurun_out/sweep_wgrad.log
