set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -m gpu > gpurun_out/t_kern.log 2>&1 || { tail -40 gpurun_out/t_kern.log; exit 1; }
tail -2 gpurun_out/t_kern.log
TILES=-1,40,41,42,43 ROUNDS=3 timeout -k 10 600 python -u tools/conv_tile_sweep.py > gpurun_out/sweep_w8.log 2>&1 || { tail -30 gpurun_out/sweep_w8.log; exit 1; }
cat gpurun_out/sweep_w8.log
