#!/bin/bash
# device JPEG decode co-running cost per kernel variant and decode-stream priority
set -o pipefail
mkdir -p gpurun_out/r6
for c in 256x10 256x11; do
  timeout -k 10 300 python -u tools/decode_overlap_bench.py --cfg $c >> gpurun_out/r6/r6_s24_decode_overlap.log 2>&1 || exit 1
done
timeout -k 10 300 python -u tools/decode_overlap_bench.py --cfg 256x10 --low-priority 1 >> gpurun_out/r6/r6_s24_decode_overlap.log 2>&1
