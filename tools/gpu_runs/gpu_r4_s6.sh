#!/bin/bash
# Round 4: Inception-v3 step timeline with the sibling merge on, 8 concurrent per-rank ImageNet pipelines,
# hipGraph scratch-growth safety tests, CU-contention A/B (reserved CUs vs a comm-like co-resident kernel).
set -o pipefail
mkdir -p gpurun_out/r4
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_fused_ops_gpu.py -k "merged_head_forward" > gpurun_out/r4/pytest_mergedfwd.log 2>&1
echo "merged fwd tests rc=$?"; grep -E "PASS|FAIL|^E  " gpurun_out/r4/pytest_mergedfwd.log | cut -c1-400 | tail -6
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
VARIANTS="base=;rsv32=rsv:32;hog16=hog:16:8;hog16r=hog:16:8,rsv:16;hog32=hog:32:8;hog32r=hog:32:8,rsv:32" STEPS=6 ROUNDS=5 timeout -k 10 400 python -u tools/ab_step.py > gpurun_out/r4/ab_hog_reserve.log 2>&1 || { tail -30 gpurun_out/r4/ab_hog_reserve.log; exit 1; }
tail -6 gpurun_out/r4/ab_hog_reserve.log
HOST_CPUS=16 timeout -k 10 400 python -u tools/multi_rank_pipeline_bench.py --ranks 8 --decoders 2 --images 4096 > gpurun_out/r4/multi_rank_pipeline.log 2>&1 || { tail -30 gpurun_out/r4/multi_rank_pipeline.log; exit 1; }
tail -5 gpurun_out/r4/multi_rank_pipeline.log
