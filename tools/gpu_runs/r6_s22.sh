#!/bin/bash
# device JPEG decode co-running with the ResNet-50 b256 training step (side stream): the step-time cost
set -o pipefail
mkdir -p gpurun_out/r6
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_jpeg.py -m gpu > gpurun_out/r6/r6_s22_pytest_jpeg.log 2>&1 &&
timeout -k 10 300 python -u tools/decode_overlap_bench.py --cfg 256x11 > gpurun_out/r6/r6_s22_decode_overlap.log 2>&1 &&
timeout -k 10 300 python -u tools/decode_overlap_bench.py --cfg 256x9 >> gpurun_out/r6/r6_s22_decode_overlap.log 2>&1 &&
timeout -k 10 300 python -u tools/decode_overlap_bench.py --cfg 64x9 >> gpurun_out/r6/r6_s22_decode_overlap.log 2>&1
