#!/bin/bash
# Round 4: strided 3x3 dgrad tile sweep (grouped parity classes) vs MIOpen: which tile the grouped launch should use.
set -o pipefail
mkdir -p gpurun_out/r4
export TMPDIR=/tmp
for t in -1 21 24 26 40 4 3 0; do
  DTM_CONV_TILE=$t STRIDED=1 timeout -k 10 200 python -u tools/conv_microbench.py > gpurun_out/r4/strided_tile$t.log 2>&1 || { tail -20 gpurun_out/r4/strided_tile$t.log; exit 1; }
  echo "tile=$t"; grep " s2 " gpurun_out/r4/strided_tile$t.log | cut -c1-200
done
