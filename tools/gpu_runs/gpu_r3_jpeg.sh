#!/bin/bash
# Split JPEG decode: GPU data tests, then sustained pipeline throughput split vs full host decode.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_data_gpu.py tests/test_jpeg.py -m gpu > gpurun_out/jpeg_gpu_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/jpeg_gpu_tests.log; exit 1; }
tail -1 gpurun_out/jpeg_gpu_tests.log
timeout -k 10 600 python -u tools/imagenet_pipeline_bench.py --images 4096 --batches 24 --warm-batches 4 --decoders 16 --mode both > gpurun_out/jpeg_pipeline.log 2>&1 || { tail -30 gpurun_out/jpeg_pipeline.log; exit 1; }
cat gpurun_out/jpeg_pipeline.log
