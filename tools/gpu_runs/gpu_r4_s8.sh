#!/bin/bash
# Round 4: grouped strided-dgrad class order (LPT) microbenchmark + conv hardware counters (two PMC passes).
set -o pipefail
mkdir -p gpurun_out/r4
export TMPDIR=/tmp
for v in 1 0 1 0; do DEC_LPT=$v STRIDED=1 NOMIO=1 timeout -k 10 200 python -u tools/conv_microbench.py > gpurun_out/r4/strided_lpt$v.log 2>&1 || { tail -20 gpurun_out/r4/strided_lpt$v.log; exit 1; }; echo "lpt=$v"; grep " s2 " gpurun_out/r4/strided_lpt$v.log | cut -c1-140; done
rm -rf gpurun_out/r4/pmc1 gpurun_out/r4/pmc2
cd /tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r4/pmc1 -o run -- python3 $GRAFT_REPO_ROOT/tools/conv_pmc_run.py > $GRAFT_REPO_ROOT/gpurun_out/r4/pmc1.log 2>&1 || { echo "pmc1 failed"; tail -20 $GRAFT_REPO_ROOT/gpurun_out/r4/pmc1.log; exit 1; }
cd /tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_WAVE_CYCLES TCC_HIT_sum TCC_MISS_sum --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r4/pmc2 -o run -- python3 $GRAFT_REPO_ROOT/tools/conv_pmc_run.py > $GRAFT_REPO_ROOT/gpurun_out/r4/pmc2.log 2>&1 || { echo "pmc2 failed"; tail -20 $GRAFT_REPO_ROOT/gpurun_out/r4/pmc2.log; exit 1; }
cd $GRAFT_REPO_ROOT
python3 tools/pmc_summary.py $(find gpurun_out/r4/pmc1 -name "*counter_collection.csv" | head -1) > gpurun_out/r4/pmc1_summary.txt 2>&1
python3 tools/pmc_summary.py $(find gpurun_out/r4/pmc2 -name "*counter_collection.csv" | head -1) > gpurun_out/r4/pmc2_summary.txt 2>&1
head -60 gpurun_out/r4/pmc1_summary.txt
rm -rf gpurun_out/r4/pmc1 gpurun_out/r4/pmc2
timeout -k 10 300 python -u tools/aten_sites.py --model inception_v3_slim_old --dispatch > gpurun_out/r4/aten_sites_inception.txt 2>&1 || { tail -20 gpurun_out/r4/aten_sites_inception.txt; exit 1; }
head -40 gpurun_out/r4/aten_sites_inception.txt | cut -c1-200
