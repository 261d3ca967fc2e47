#!/bin/bash
# Round 6 session 3: library GEMM (hipBLASLt via torch.matmul) on the conv-equivalent GEMM shapes vs our conv tiles.
set -o pipefail
mkdir -p gpurun_out/r6
TILES=-1,40,41,21 timeout -k 10 300 python -u tools/gemm_ref_bench.py > gpurun_out/r6/r6_s3_gemm_ref.log 2>&1 || { tail -20 gpurun_out/r6/r6_s3_gemm_ref.log; exit 1; }
cat gpurun_out/r6/r6_s3_gemm_ref.log
