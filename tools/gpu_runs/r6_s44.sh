#!/bin/bash
# round-6 occupancy launch bounds of the register-staged conv tiles on Inception-v3 / VGG-16 (tuned on ResNet-50):
# default (aocc = nocc = 2) vs the round-5 launches (0), captured benches alternated
set -o pipefail
mkdir -p gpurun_out/r6
for m in inception_v3_slim_old vgg_16; do
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --model $m --steps 30 --warmup 5 > gpurun_out/r6/r6_s44_${m}_def_$i.log 2>&1 || exit 1
  DTM_ACT_OCC=0 DTM_NT_OCC=0 timeout -k 10 200 python -u bench.py --model $m --steps 30 --warmup 5 > gpurun_out/r6/r6_s44_${m}_occ0_$i.log 2>&1 || exit 1
  echo "$m round $i: default $(tail -1 gpurun_out/r6/r6_s44_${m}_def_$i.log | python -c 'import json,sys; print(json.loads(sys.stdin.read())["value"])') occ0 $(tail -1 gpurun_out/r6/r6_s44_${m}_occ0_$i.log | python -c 'import json,sys; print(json.loads(sys.stdin.read())["value"])')"
done
done
