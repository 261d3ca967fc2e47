#!/bin/bash
# Grouped stride-decomposed dgrad launch + dgrad-epilogue BN-apply backward for stride-2 unit outputs:
# numerics (new + neighbouring GPU tests), ResNet-50 same-process A/B, conv table.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_fused_ops_gpu.py tests/test_kernels_gpu.py > gpurun_out/dgrp_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/dgrp_tests.log; exit 1; }
tail -1 gpurun_out/dgrp_tests.log
VARIANTS="new=;nogrp=dgrp:0;nobnst=bnst:0;old=dgrp:0,bnst:0;s75=scu:75" ROUNDS=5 timeout -k 10 400 python -u tools/ab_step.py > gpurun_out/r3_ab_dgrp_bnst.log 2>&1 || { tail -30 gpurun_out/r3_ab_dgrp_bnst.log; exit 1; }
tail -5 gpurun_out/r3_ab_dgrp_bnst.log
STRIDED=1 timeout -k 10 300 python -u tools/conv_microbench.py > gpurun_out/r3_conv_table_strided_grp.txt 2>&1 || { tail -20 gpurun_out/r3_conv_table_strided_grp.txt; exit 1; }
cat gpurun_out/r3_conv_table_strided_grp.txt
