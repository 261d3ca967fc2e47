#!/bin/bash
# device entropy decode with checkpoint merges in the re-decode passes: numerics, throughput, co-running cost
set -o pipefail
mkdir -p gpurun_out/r6
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 120 --timeout-method thread tests/test_jpeg.py tests/test_data_gpu.py -m gpu -k "jpeg or decode" > gpurun_out/r6/r6_s28_pytest_jpeg.log 2>&1 || { tail -30 gpurun_out/r6/r6_s28_pytest_jpeg.log; exit 1; }
tail -1 gpurun_out/r6/r6_s28_pytest_jpeg.log
timeout -k 10 300 python -u tools/jpeg_gpu_bench.py --images 768 --cfg 256x10 256x11 128x10 > gpurun_out/r6/r6_s28_jpeg_bench768.log 2>&1 &&
timeout -k 10 300 python -u tools/jpeg_gpu_bench.py --images 256 --cfg 256x10 > gpurun_out/r6/r6_s28_jpeg_bench256.log 2>&1 &&
timeout -k 10 300 python -u tools/decode_overlap_bench.py --cfg 256x10 > gpurun_out/r6/r6_s28_decode_overlap.log 2>&1
grep -hv amdgpu gpurun_out/r6/r6_s28_jpeg_bench768.log gpurun_out/r6/r6_s28_jpeg_bench256.log gpurun_out/r6/r6_s28_decode_overlap.log
