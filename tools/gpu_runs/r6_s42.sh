#!/bin/bash
# after restricting the stem BN-fused pipelined wgrad tile to K > 32: Inception stem sweep + captured bench
set -o pipefail
mkdir -p gpurun_out/r6
INC=1 TILES=-1 WTILES=-1,6 ROUNDS=5 timeout -k 10 300 python -u tools/stem_sweep.py > gpurun_out/r6/r6_s42_stem_inception.log 2>&1 || exit 1
grep "wg+bn" gpurun_out/r6/r6_s42_stem_inception.log
TILES=-1 WTILES=-1,15:2,6 ROUNDS=3 timeout -k 10 300 python -u tools/stem_sweep.py > gpurun_out/r6/r6_s42_stem_resnet.log 2>&1 || exit 1
grep "wg+bn" gpurun_out/r6/r6_s42_stem_resnet.log
for i in 1 2; do
timeout -k 10 200 python -u bench.py --model inception_v3_slim_old --steps 20 --warmup 5 > gpurun_out/r6/r6_s42_bench_inception_$i.log 2>&1 || exit 1
tail -1 gpurun_out/r6/r6_s42_bench_inception_$i.log | cut -c1-160
done
