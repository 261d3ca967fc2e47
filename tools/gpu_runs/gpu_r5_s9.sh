#!/bin/bash
# Round 5 session 9: where does the one-rank RCCL data-parallel path hang?  Probes from plain to the bench's settings.
set -o pipefail
mkdir -p gpurun_out/r5
export TMPDIR=/tmp
PROBE_TIMING=0 PROBE_HIPRIO=0 timeout -k 10 100 python -u tools/rccl_probe.py 2>&1 | tee gpurun_out/r5/r5_rccl_probe_plain.log &&
PROBE_TIMING=1 PROBE_HIPRIO=0 timeout -k 10 100 python -u tools/rccl_probe.py 2>&1 | tee gpurun_out/r5/r5_rccl_probe_timing.log &&
PROBE_TIMING=1 PROBE_HIPRIO=1 timeout -k 10 100 python -u tools/rccl_probe.py 2>&1 | tee gpurun_out/r5/r5_rccl_probe_default.log
echo "rc=$?"
