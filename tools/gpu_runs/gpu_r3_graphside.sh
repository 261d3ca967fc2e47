#!/bin/bash
# Per-shape conv table (ours vs MIOpen, fwd / dgrad / wgrad, ResNet-50 shapes at B=256, stem dgrad excluded).
# (The hipGraph-captured side-stream A/B this script first ran faulted on replay; the capture path now stays
#  single-stream: profiles/ab/README.md, round 3.)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/conv_microbench.py > gpurun_out/r3_conv_table_vs_miopen.txt 2>&1 || { tail -20 gpurun_out/r3_conv_table_vs_miopen.txt; exit 1; }
tail -3 gpurun_out/r3_conv_table_vs_miopen.txt
