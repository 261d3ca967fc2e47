#!/bin/bash
# Round 4: act-dgrad LDS tiles + block-output dgrad stream-side kernel (numerics, A/B, bench, kernel stats, tile
# decisions) and the 2-step DP checks of the sibling merge.
set -o pipefail
mkdir -p gpurun_out/r4
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_dgrad_decomposition.py -k "act_dgrad or bnout or decomposed or pipelined_tiles" > gpurun_out/r4/pytest_s3.log 2>&1 || { tail -30 gpurun_out/r4/pytest_s3.log; exit 1; }
tail -2 gpurun_out/r4/pytest_s3.log
timeout -k 10 300 python -u tools/dp_grad_diag.py resnet_v1_50 DTM_SIBLING_GROUP=1 --steps 2 > gpurun_out/r4/diag_resnet_sib_2steps.log 2>&1 || { tail -30 gpurun_out/r4/diag_resnet_sib_2steps.log; exit 1; }
grep -E "RESULT|tensors differ" gpurun_out/r4/diag_resnet_sib_2steps.log
DTM_SIBLING_GROUP=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_distributed.py -k "two_ranks_hip_kernels" > gpurun_out/r4/pytest_dp_r3test_sib.log 2>&1
echo "r3-style 2-step DP test with sibling: rc=$?"
tail -3 gpurun_out/r4/pytest_dp_r3test_sib.log | cut -c1-300
VARIANTS="base=;noside=sside:0;noalds=alds:0;neither=sside:0,alds:0" STEPS=6 ROUNDS=5 timeout -k 10 400 python -u tools/ab_step.py > gpurun_out/r4/ab_sside_alds.log 2>&1 || { tail -30 gpurun_out/r4/ab_sside_alds.log; exit 1; }
tail -4 gpurun_out/r4/ab_sside_alds.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r4/bench_resnet_s3.log 2>&1 || { tail -30 gpurun_out/r4/bench_resnet_s3.log; exit 1; }
tail -1 gpurun_out/r4/bench_resnet_s3.log | cut -c1-200
DTM_TILE_LOG=1 timeout -k 10 200 python -u bench.py --steps 1 --warmup 1 > gpurun_out/r4/tilelog_resnet.out 2> gpurun_out/r4/tilelog_resnet.err || { tail -30 gpurun_out/r4/tilelog_resnet.err; exit 1; }
rm -rf gpurun_out/r4/prof_s3
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r4/prof_s3 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 3 > $GRAFT_REPO_ROOT/gpurun_out/r4/prof_s3.log 2>&1 || { echo "prof failed"; tail -30 $GRAFT_REPO_ROOT/gpurun_out/r4/prof_s3.log; exit 1; }
cd $GRAFT_REPO_ROOT
f=$(find gpurun_out/r4/prof_s3 -name "*kernel_stats.csv" | head -1)
cp "$f" gpurun_out/r4/r4_s3_kernel_stats.csv
t=$(find gpurun_out/r4/prof_s3 -name "*kernel_trace.csv" | head -1)
python3 tools/step_timeline.py "$t" > gpurun_out/r4/r4_s3_timeline.txt
tail -1 gpurun_out/r4/r4_s3_timeline.txt
rm -rf gpurun_out/r4/prof_s3
