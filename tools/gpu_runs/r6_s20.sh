#!/bin/bash
# device entropy decode: block context in registers, inline slow path, refill wait moved to the next refill
set -o pipefail
mkdir -p gpurun_out/r6
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 120 --timeout-method thread tests/test_jpeg.py -m gpu > gpurun_out/r6/r6_s20_pytest_jpeg.log 2>&1 &&
timeout -k 10 200 python -u tools/jpeg_gpu_bench.py --images 128 --overlap -1 > gpurun_out/r6/r6_s20_jpeg_bench.log 2>&1 &&
timeout -k 10 200 python -u tools/jpeg_gpu_bench.py --images 768 --overlap -1 2048 > gpurun_out/r6/r6_s20_jpeg_bench768.log 2>&1
