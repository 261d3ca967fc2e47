#!/bin/bash
# device entropy decode: threads-per-image x lookup-bits variants, warm-up overlap
set -o pipefail
mkdir -p gpurun_out/r6
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 120 --timeout-method thread tests/test_jpeg.py -m gpu > gpurun_out/r6/r6_s21_pytest_jpeg.log 2>&1 &&
timeout -k 10 400 python -u tools/jpeg_gpu_bench.py --images 768 --overlap -1 4096 --cfg 256x11 256x9 128x10 64x11 64x9 > gpurun_out/r6/r6_s21_jpeg_bench768.log 2>&1
