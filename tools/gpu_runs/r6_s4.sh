#!/bin/bash
# Round 6 session 4: PMC passes of the w8 (tile 40 / wgrad 12) and ping-pong (41 / 13) 256x256 kernels on the
# 7x7 3x3 512 and 14x14 3x3 256 ResNet-50 layers (fwd, dgrad, wgrad): where the main loops wait.
set -o pipefail
mkdir -p gpurun_out/r6/pmc4
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp
for S in 7_512_512_3 14_256_256_3; do
for T in 40 41; do
  PP=0; [ $T = 41 ] && PP=1
  ONLY=$S NOMIO=1 B=256 DTM_CONV_TILE=$T DTM_PP=$PP timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES --output-format csv -d $R/gpurun_out/r6/pmc4/${S}_$T -o run -- python3 $R/tools/conv_microbench.py > $R/gpurun_out/r6/pmc4/${S}_$T.log 2>&1 || { echo "pmc $S $T failed"; tail -5 $R/gpurun_out/r6/pmc4/${S}_$T.log; exit 1; }
  ONLY=$S NOMIO=1 B=256 DTM_CONV_TILE=$T DTM_PP=$PP timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_WAVES --output-format csv -d $R/gpurun_out/r6/pmc4/${S}_${T}b -o run -- python3 $R/tools/conv_microbench.py > $R/gpurun_out/r6/pmc4/${S}_${T}b.log 2>&1 || { echo "pmc2 $S $T failed"; tail -5 $R/gpurun_out/r6/pmc4/${S}_${T}b.log; exit 1; }
done
done
cd $R
for f in $(find gpurun_out/r6/pmc4 -name "*counter_collection.csv" | sort); do echo "== $f"; python3 tools/pmc_summary.py "$f"; done > gpurun_out/r6/r6_s4_pmc_summary.txt
find gpurun_out/r6/pmc4 -name "*.csv" -delete
cat gpurun_out/r6/r6_s4_pmc_summary.txt | head -120
