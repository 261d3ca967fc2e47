#!/bin/bash
# Round 4: merged sibling-head forward tile sweep on the Inception-v3 head shapes (batch 128).
set -o pipefail
mkdir -p gpurun_out/r4
export TMPDIR=/tmp
for t in -1 4 3 0 21 24 26 40; do
  DTM_CONV_TILE=$t timeout -k 10 120 python -u tools/split_tile_sweep.py > gpurun_out/r4/split_tile$t.log 2>&1 || { tail -20 gpurun_out/r4/split_tile$t.log; exit 1; }
  echo "== tile $t"; grep -v amdgpu.ids gpurun_out/r4/split_tile$t.log
done
