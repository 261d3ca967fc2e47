#!/bin/bash
# Round 4: Inception-v3 step timeline with the sibling merge on, 8 concurrent per-rank ImageNet pipelines,
# hipGraph scratch-growth safety tests, CU-contention A/B (reserved CUs vs a comm-like co-resident kernel).
set -o pipefail
mkdir -p gpurun_out/r4
export TMPDIR=/tmp
rm -rf gpurun_out/r4/prof_inc
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r4/prof_inc -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --model inception_v3_slim_old --graph 0 --steps 3 --warmup 2 > $GRAFT_REPO_ROOT/gpurun_out/r4/prof_inc.log 2>&1 || { echo "prof failed"; tail -30 $GRAFT_REPO_ROOT/gpurun_out/r4/prof_inc.log; exit 1; }
cd $GRAFT_REPO_ROOT
f=$(find gpurun_out/r4/prof_inc -name "*kernel_stats.csv" | head -1)
cp "$f" gpurun_out/r4/r4_inception_kernel_stats.csv
t=$(find gpurun_out/r4/prof_inc -name "*kernel_trace.csv" | head -1)
python3 tools/step_timeline.py "$t" > gpurun_out/r4/r4_inception_timeline.txt
tail -1 gpurun_out/r4/r4_inception_timeline.txt
rm -rf gpurun_out/r4/prof_inc
timeout -k 10 300 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_engine.py -m gpu -k "scratch or larger or graph" > gpurun_out/r4/pytest_graphsafe.log 2>&1
echo "graph-safety tests rc=$?"; tail -2 gpurun_out/r4/pytest_graphsafe.log
VARIANTS="base=;hog16=hog:16:8;hog16r=hog:16:8,rsv:16;hog32=hog:32:8;hog32r=hog:32:8,rsv:32" STEPS=6 ROUNDS=5 timeout -k 10 400 python -u tools/ab_step.py > gpurun_out/r4/ab_hog_reserve.log 2>&1 || { tail -30 gpurun_out/r4/ab_hog_reserve.log; exit 1; }
tail -6 gpurun_out/r4/ab_hog_reserve.log
HOST_CPUS=16 timeout -k 10 400 python -u tools/multi_rank_pipeline_bench.py --ranks 8 --decoders 2 --images 4096 > gpurun_out/r4/multi_rank_pipeline.log 2>&1 || { tail -30 gpurun_out/r4/multi_rank_pipeline.log; exit 1; }
tail -5 gpurun_out/r4/multi_rank_pipeline.log
for v in 1 0 1 0; do DEC_LPT=$v STRIDED=1 timeout -k 10 200 python -u tools/conv_microbench.py > gpurun_out/r4/strided_lpt$v.log 2>&1 || { tail -20 gpurun_out/r4/strided_lpt$v.log; exit 1; }; echo "lpt=$v"; grep " s2 " gpurun_out/r4/strided_lpt$v.log | cut -c1-140; done
rm -rf gpurun_out/r4/pmc1 gpurun_out/r4/pmc2
cd /tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r4/pmc1 -o run -- python3 $GRAFT_REPO_ROOT/tools/conv_pmc_run.py > $GRAFT_REPO_ROOT/gpurun_out/r4/pmc1.log 2>&1 || { echo "pmc1 failed"; tail -20 $GRAFT_REPO_ROOT/gpurun_out/r4/pmc1.log; exit 1; }
cd /tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_WAVE_CYCLES TCC_HIT_sum TCC_MISS_sum --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r4/pmc2 -o run -- python3 $GRAFT_REPO_ROOT/tools/conv_pmc_run.py > $GRAFT_REPO_ROOT/gpurun_out/r4/pmc2.log 2>&1 || { echo "pmc2 failed"; tail -20 $GRAFT_REPO_ROOT/gpurun_out/r4/pmc2.log; exit 1; }
cd $GRAFT_REPO_ROOT
python3 tools/pmc_summary.py $(find gpurun_out/r4/pmc1 -name "*counter_collection.csv" | head -1) > gpurun_out/r4/pmc1_summary.txt 2>&1
python3 tools/pmc_summary.py $(find gpurun_out/r4/pmc2 -name "*counter_collection.csv" | head -1) > gpurun_out/r4/pmc2_summary.txt 2>&1
head -60 gpurun_out/r4/pmc1_summary.txt
rm -rf gpurun_out/r4/pmc1 gpurun_out/r4/pmc2
