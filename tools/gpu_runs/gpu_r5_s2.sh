#!/bin/bash
# Round 5 session 2: the whole GPU suite (new: Inception-v3 whole-step numerics, distinct-batch DP gradients, feature
# registry), roofline passes (read bytes by request size + MFMA MOPS; write bytes + DRAM read requests), conv shape
# log trace, Inception kernel trace.
set -o pipefail
mkdir -p gpurun_out/r5
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 780 python -u -m pytest -v -s --timeout 400 --timeout-method thread tests -m gpu > gpurun_out/r5/r5_s2_pytest_gpu.log 2>&1
rc=$?; echo "gpu suite rc=$rc"; grep -E "FAILED|ERROR" gpurun_out/r5/r5_s2_pytest_gpu.log | head -20; tail -1 gpurun_out/r5/r5_s2_pytest_gpu.log
case $rc in 0|1) ;; *) exit $rc ;; esac
cd /tmp
timeout -k 10 240 rocprofv3 --pmc TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum SQ_INSTS_VALU_MFMA_MOPS_BF16 --kernel-trace --output-format csv -d $R/gpurun_out/r5/pmc_a -o a -- python3 $R/bench.py --steps 3 --warmup 2 > $R/gpurun_out/r5/pmc_a.log 2>&1 || { echo "pass a failed"; tail -20 $R/gpurun_out/r5/pmc_a.log; exit 1; }
timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE TCC_EA0_RDREQ_DRAM_sum --kernel-trace --output-format csv -d $R/gpurun_out/r5/pmc_b -o b -- python3 $R/bench.py --steps 3 --warmup 2 > $R/gpurun_out/r5/pmc_b.log 2>&1 || { echo "pass b failed"; tail -20 $R/gpurun_out/r5/pmc_b.log; exit 1; }
cd $R
python3 tools/roofline_report.py 3 gpurun_out/r5/pmc_a/a_counter_collection.csv gpurun_out/r5/pmc_b/b_counter_collection.csv --top 50 > gpurun_out/r5/r5_resnet50_roofline.txt 2>&1 || { tail -5 gpurun_out/r5/r5_resnet50_roofline.txt; exit 1; }
head -3 gpurun_out/r5/r5_resnet50_roofline.txt
cd /tmp
DTM_TILE_LOG=1 timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/r5/trace_tl -o t -- python3 $R/bench.py --steps 2 --warmup 1 > $R/gpurun_out/r5/trace_tl.log 2>&1 || { echo "tile-log trace failed"; tail -20 $R/gpurun_out/r5/trace_tl.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r5/trace_inc -o t -- python3 $R/bench.py --model inception_v3_slim_old --steps 3 --warmup 3 > $R/gpurun_out/r5/trace_inc.log 2>&1 || { echo "inception trace failed"; tail -20 $R/gpurun_out/r5/trace_inc.log; exit 1; }
cd $R
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r5/r5_s2_bench_resnet.log 2>&1 && tail -1 gpurun_out/r5/r5_s2_bench_resnet.log | cut -c1-150
echo done
