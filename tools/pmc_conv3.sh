#!/bin/bash
# PMC counters of the compute-bound conv kernels (3x3 at 14x14 / 7x7 / 28x28): where the main loop waits.
set -o pipefail
mkdir -p gpurun_out/pmc3
export TMPDIR=/tmp
cd /tmp
for S in 14_256_256_3 7_512_512_3 28_128_128_3; do
  ONLY=$S NOMIO=1 B=256 timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/pmc3/$S -o run -- python3 $GRAFT_REPO_ROOT/tools/conv_microbench.py > $GRAFT_REPO_ROOT/gpurun_out/pmc3/$S.log 2>&1 || { echo "pmc $S failed"; tail -5 $GRAFT_REPO_ROOT/gpurun_out/pmc3/$S.log; exit 1; }
done
cd $GRAFT_REPO_ROOT
for f in $(find gpurun_out/pmc3 -name "*counter_collection.csv"); do echo "== $f"; python3 tools/pmc_summary.py "$f"; done
