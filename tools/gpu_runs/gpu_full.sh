set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1 || { tail -20 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log | cut -c1-260
timeout -k 10 300 python bench.py --model vgg_16 --gpus 2 --dist-backend gloo --steps 3 --warmup 2 > gpurun_out/bench_vgg_gloo2.log 2>&1 || { tail -20 gpurun_out/bench_vgg_gloo2.log; exit 1; }
tail -1 gpurun_out/bench_vgg_gloo2.log
timeout -k 10 300 python bench.py --model inception_v3_slim_old --steps 10 --warmup 3 > gpurun_out/bench_incep.log 2>&1 || { tail -20 gpurun_out/bench_incep.log; exit 1; }
tail -1 gpurun_out/bench_incep.log | cut -c1-260
