#!/bin/bash
# same-box ResNet-50 bench: the s25 checkpoint (6c590ec, build/ab_base) vs the current tree, alternated twice
set -o pipefail
mkdir -p gpurun_out/r6
R=$GRAFT_REPO_ROOT
for i in 1 2; do
  (cd build/ab_base && timeout -k 10 200 python -u bench.py --steps 30 --warmup 5) > gpurun_out/r6/r6_s36_base_$i.log 2>&1 || exit 1
  timeout -k 10 200 python -u bench.py --steps 30 --warmup 5 > gpurun_out/r6/r6_s36_head_$i.log 2>&1 || exit 1
  echo "round $i: base $(tail -1 gpurun_out/r6/r6_s36_base_$i.log | python -c 'import json,sys; print(json.loads(sys.stdin.read())["value"])') head $(tail -1 gpurun_out/r6/r6_s36_head_$i.log | python -c 'import json,sys; print(json.loads(sys.stdin.read())["value"])')"
done
