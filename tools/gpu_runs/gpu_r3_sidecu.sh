#!/bin/bash
# Side-stream weight-gradient split-K sizing (percent of the CUs the split policy fills) A/B on ResNet-50, then the
# per-shape conv table vs MIOpen.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
VARIANTS="s100=scu:100;s75=scu:75;s50=scu:50;s35=scu:35" ROUNDS=5 timeout -k 10 400 python -u tools/ab_step.py > gpurun_out/r3_ab_side_cus.log 2>&1 || { tail -30 gpurun_out/r3_ab_side_cus.log; exit 1; }
tail -4 gpurun_out/r3_ab_side_cus.log
timeout -k 10 400 python -u tools/conv_microbench.py > gpurun_out/r3_conv_table_vs_miopen.txt 2>&1 || { tail -20 gpurun_out/r3_conv_table_vs_miopen.txt; exit 1; }
tail -3 gpurun_out/r3_conv_table_vs_miopen.txt
