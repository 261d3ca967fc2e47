#!/bin/bash
# Per-shape conv table (ours vs MIOpen fwd / dgrad / wgrad) over the ResNet-50 shapes at B=256, then
# eager-vs-hipGraph whole-step A/B for ResNet-50 and Inception-v3.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/conv_microbench.py > gpurun_out/conv_table.txt 2>&1 || { tail -20 gpurun_out/conv_table.txt; exit 1; }
cat gpurun_out/conv_table.txt
if [ -n "$GRAPH_AB" ]; then bash tools/gpu_runs/gpu_graph_ab.sh || exit 1; fi
