#!/bin/bash
# Round 4: merged sibling-head forward vs per-head with a fixed gradient backpropagated from the first / second mixed
# block's output only (Inception-v3, batch 2 and 4) - the merged path without the whole random-init net's drift.
set -o pipefail
mkdir -p gpurun_out/r4
export TMPDIR=/tmp
for blk in mixed_35x35x256a mixed_35x35x288a mixed_17x17x768a; do
  for b in 4; do
    timeout -k 10 300 python -u tools/diag_sibfwd.py --batch $b --block $blk > gpurun_out/r4/diag_sibfwd_${blk}_b$b.log 2>&1 || { tail -30 gpurun_out/r4/diag_sibfwd_${blk}_b$b.log; exit 1; }
    echo "== $blk batch $b"; grep -v amdgpu.ids gpurun_out/r4/diag_sibfwd_${blk}_b$b.log | grep -v amdgpu
  done
done
