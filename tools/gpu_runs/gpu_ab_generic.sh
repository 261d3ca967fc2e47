#!/bin/bash
# Same-process whole-step A/B (tools/ab_step.py) with $VARIANTS, output to gpurun_out/$OUT (default ab.log);
# optional GEMM yardstick first (GEMM=1).
set -o pipefail
mkdir -p gpurun_out
if [ -n "$GEMM" ]; then timeout -k 10 120 python tools/gemm_probe.py > gpurun_out/gemm_probe.txt 2>&1 || { tail gpurun_out/gemm_probe.txt; exit 1; }; cat gpurun_out/gemm_probe.txt; fi
timeout -k 10 ${TLIM:-420} python -u tools/ab_step.py > gpurun_out/${OUT:-ab.log} 2>&1 || { tail -20 gpurun_out/${OUT:-ab.log}; exit 1; }
tail -${TAILN:-3} gpurun_out/${OUT:-ab.log}
