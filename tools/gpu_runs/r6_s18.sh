#!/bin/bash
# device entropy decode: numerics tests + throughput
set -o pipefail
mkdir -p gpurun_out/r6
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 120 --timeout-method thread tests/test_jpeg.py -m gpu > gpurun_out/r6/r6_s18_pytest_jpeg.log 2>&1 &&
timeout -k 10 200 python -u tools/jpeg_gpu_bench.py --images 128 > gpurun_out/r6/r6_s18_jpeg_bench.log 2>&1
