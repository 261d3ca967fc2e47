set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_data_gpu.py -m gpu > gpurun_out/t_data.log 2>&1 || { tail -40 gpurun_out/t_data.log; exit 1; }
tail -2 gpurun_out/t_data.log
timeout -k 10 500 python -u tools/imagenet_pipeline_bench.py --images 3072 --decoders 16 --host > gpurun_out/imnet_pipe.log 2>&1 || { tail -20 gpurun_out/imnet_pipe.log; exit 1; }
cat gpurun_out/imnet_pipe.log
