#!/bin/bash
# device entropy decode with LDS-staged phases: numerics, pipeline, throughput, co-running cost, box host CPU cost
set -o pipefail
mkdir -p gpurun_out/r6
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 120 --timeout-method thread tests/test_jpeg.py tests/test_data_gpu.py -m gpu -k "jpeg or decode" > gpurun_out/r6/r6_s23_pytest_jpeg.log 2>&1 &&
timeout -k 10 300 python -u tools/jpeg_gpu_bench.py --images 768 --cfg 256x11 256x10 256x9 128x10 128x9 64x9 > gpurun_out/r6/r6_s23_jpeg_bench768.log 2>&1 &&
timeout -k 10 300 python -u tools/jpeg_gpu_bench.py --images 256 --cfg 256x11 256x9 128x9 > gpurun_out/r6/r6_s23_jpeg_bench256.log 2>&1 &&
timeout -k 10 300 python -u tools/decode_overlap_bench.py --cfg 256x9 > gpurun_out/r6/r6_s23_decode_overlap.log 2>&1 &&
timeout -k 10 300 python -u tools/decode_overlap_bench.py --cfg 128x9 >> gpurun_out/r6/r6_s23_decode_overlap.log 2>&1 &&
timeout -k 10 300 python -u tools/decode_cpu_cost.py --images 256 > gpurun_out/r6/r6_decode_cpu_cost_box.log 2>&1
