#!/bin/bash
# Inception-v3 step with the direct 3x3 weight gradient for the stem's 32-channel 3x3s (wdir) vs the register-staged
# implicit-GEMM tiles; captured bench after
set -o pipefail
mkdir -p gpurun_out/r6
MODEL=inception_v3_slim_old VARIANTS="base=;nowdir=wdir:0" ROUNDS=5 timeout -k 10 500 python -u tools/ab_step.py > gpurun_out/r6/r6_s34_ab_wdir_inception.log 2>&1 || { tail -20 gpurun_out/r6/r6_s34_ab_wdir_inception.log; exit 1; }
tail -3 gpurun_out/r6/r6_s34_ab_wdir_inception.log
timeout -k 10 200 python -u bench.py --model inception_v3_slim_old --steps 20 --warmup 5 > gpurun_out/r6/r6_s34_bench_inception.log 2>&1 || exit 1
tail -1 gpurun_out/r6/r6_s34_bench_inception.log | cut -c1-200
DTM_WGRAD_DIRECT=0 DTM_DIRECT_CT32=0 timeout -k 10 200 python -u bench.py --model inception_v3_slim_old --steps 20 --warmup 5 > gpurun_out/r6/r6_s34_bench_inception_old.log 2>&1 || exit 1
tail -1 gpurun_out/r6/r6_s34_bench_inception_old.log | cut -c1-200
