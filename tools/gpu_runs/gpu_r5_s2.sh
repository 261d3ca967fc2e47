#!/bin/bash
# Round 5 session 2: Inception-v3 whole-step numerics (trajectory / teacher-forced / noise floor), roofline passes
# (read bytes by request size + MFMA MOPS; write bytes + DRAM read requests), conv shape log for the trace.
set -o pipefail
mkdir -p gpurun_out/r5
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 600 --timeout-method thread tests/test_trajectory_inception_gpu.py > gpurun_out/r5/r5_s2_pytest_inception_numerics.log 2>&1
rc=$?; tail -30 gpurun_out/r5/r5_s2_pytest_inception_numerics.log | cut -c1-300
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
cd /tmp
timeout -k 10 240 rocprofv3 --pmc TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum SQ_INSTS_VALU_MFMA_MOPS_BF16 --kernel-trace --output-format csv -d $R/gpurun_out/r5/pmc_a -o a -- python3 $R/bench.py --steps 3 --warmup 2 > $R/gpurun_out/r5/pmc_a.log 2>&1 || { echo "pass a failed"; tail -20 $R/gpurun_out/r5/pmc_a.log; exit 1; }
timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE TCC_EA0_RDREQ_DRAM_sum --kernel-trace --output-format csv -d $R/gpurun_out/r5/pmc_b -o b -- python3 $R/bench.py --steps 3 --warmup 2 > $R/gpurun_out/r5/pmc_b.log 2>&1 || { echo "pass b failed"; tail -20 $R/gpurun_out/r5/pmc_b.log; exit 1; }
cd $R
python3 tools/roofline_report.py 3 gpurun_out/r5/pmc_a/a_counter_collection.csv gpurun_out/r5/pmc_b/b_counter_collection.csv --top 50 > gpurun_out/r5/r5_resnet50_roofline.txt 2>&1 || { tail -5 gpurun_out/r5/r5_resnet50_roofline.txt; exit 1; }
head -3 gpurun_out/r5/r5_resnet50_roofline.txt
cd /tmp
DTM_TILE_LOG=1 timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/r5/trace_tl -o t -- python3 $R/bench.py --steps 2 --warmup 1 > $R/gpurun_out/r5/trace_tl.log 2>&1 || { echo "tile-log trace failed"; tail -20 $R/gpurun_out/r5/trace_tl.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r5/trace_inc -o t -- python3 $R/bench.py --model inception_v3_slim_old --steps 3 --warmup 3 > $R/gpurun_out/r5/trace_inc.log 2>&1 || { echo "inception trace failed"; tail -20 $R/gpurun_out/r5/trace_inc.log; exit 1; }
echo done
