#!/bin/bash
# same-box Inception-v3 captured bench: before (06aca7f, build/ab_base) vs after the stem-tile fix, alternated twice
set -o pipefail
mkdir -p gpurun_out/r6
for i in 1 2; do
  (cd build/ab_base && timeout -k 10 200 python -u bench.py --model inception_v3_slim_old --steps 30 --warmup 5) > gpurun_out/r6/r6_s43_base_$i.log 2>&1 || exit 1
  timeout -k 10 200 python -u bench.py --model inception_v3_slim_old --steps 30 --warmup 5 > gpurun_out/r6/r6_s43_head_$i.log 2>&1 || exit 1
  echo "round $i: base $(tail -1 gpurun_out/r6/r6_s43_base_$i.log | python -c 'import json,sys; print(json.loads(sys.stdin.read())["value"])') head $(tail -1 gpurun_out/r6/r6_s43_head_$i.log | python -c 'import json,sys; print(json.loads(sys.stdin.read())["value"])')"
done
