#!/bin/bash
# Stem forward as a persistent stream (+ SIDE-less stream epilogues), side-stream weight gradients:
# numerics, whole-step A/B, per-kernel profile.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_fused_ops_gpu.py tests/test_kernels_gpu.py -k "stem or stream or conv or side" > gpurun_out/stem_tests.log 2>&1 || { echo "stem tests failed"; tail -40 gpurun_out/stem_tests.log; exit 1; }
tail -1 gpurun_out/stem_tests.log
VARIANTS="ring3=sstr:1;ring2=sstr:2;off=sstr:0;wgs=wgs:1" ROUNDS=5 timeout -k 10 400 python -u tools/ab_step.py > gpurun_out/stem_step.log 2>&1 || { tail -30 gpurun_out/stem_step.log; exit 1; }
tail -5 gpurun_out/stem_step.log
for v in 1 0; do
VARIANTS="s=sstr:$v" ROUNDS=1 STEPS=3 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_stem$v -o run -- python3 -u tools/ab_step.py > gpurun_out/stem_prof$v.log 2>&1 || { tail -30 gpurun_out/stem_prof$v.log; exit 1; }
f=$(ls gpurun_out/prof_stem$v/run_kernel_stats.csv gpurun_out/prof_stem$v/*/run_kernel_stats.csv 2>/dev/null | head -1)
echo "== sstr=$v $f"; python3 tools/prof_summary.py "$f" 5 40 | grep -i "total\|stream\|pipe_kernel<128, 64"
done
