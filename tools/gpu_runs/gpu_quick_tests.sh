set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_activation_gpu.py tests/test_kernels_gpu.py tests/test_zoo_gpu.py -m gpu > gpurun_out/t_act.log 2>&1 || { tail -40 gpurun_out/t_act.log; exit 1; }
tail -2 gpurun_out/t_act.log
