#!/bin/bash
# Round 4: merged sibling-head forward vs per-head, per-block gradient errors (Inception-v3, batch 2 / 4); then the
# final evidence part 2 (8-rank gloo rehearsal, ResNet-50 kernel trace).
set -o pipefail
mkdir -p gpurun_out/r4
export TMPDIR=/tmp
for b in 2 4; do
  timeout -k 10 300 python -u tools/diag_sibfwd.py --batch $b > gpurun_out/r4/diag_sibfwd_b$b.log 2>&1 || { tail -30 gpurun_out/r4/diag_sibfwd_b$b.log; exit 1; }
  cat gpurun_out/r4/diag_sibfwd_b$b.log | grep -v amdgpu.ids
done
bash tools/gpu_runs/gpu_r4_final2.sh
