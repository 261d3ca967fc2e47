#!/bin/bash
# Round 5 session 6: slab-reduction offload stream (Inception-v3) + one-launch multi-destination slab reduction:
# numerics, same-process eager A/B, captured bench with and without, kernel trace of the captured step.
set -o pipefail
mkdir -p gpurun_out/r5
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -v -s --timeout 400 --timeout-method thread tests/test_engine.py tests/test_kernels_gpu.py tests/test_fused_ops_gpu.py -m gpu -k "offload or hipgraph or wgrad_multi or sibling or finalize_direct" > gpurun_out/r5/r5_s6_pytest.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/r5/r5_s6_pytest.log | tail -5
[ $rc -eq 0 ] || exit $rc
MODEL=inception_v3_slim_old VARIANTS="base=;nooff=off:reduce_offload" STEPS=6 ROUNDS=5 timeout -k 10 400 python -u tools/ab_step.py > gpurun_out/r5/r5_ab_offload_inception.log 2>&1; tail -3 gpurun_out/r5/r5_ab_offload_inception.log
for i in 1 2; do
timeout -k 10 200 python -u bench.py --model inception_v3_slim_old --steps 20 --warmup 5 > gpurun_out/r5/r5_s6_bench_inc_off_$i.log 2>&1 && tail -1 gpurun_out/r5/r5_s6_bench_inc_off_$i.log | cut -c1-140
DTM_DISABLE=reduce_offload timeout -k 10 200 python -u bench.py --model inception_v3_slim_old --steps 20 --warmup 5 > gpurun_out/r5/r5_s6_bench_inc_nooff_$i.log 2>&1 && tail -1 gpurun_out/r5/r5_s6_bench_inc_nooff_$i.log | cut -c1-140
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r5/trace_inc2 -o t -- python3 $GRAFT_REPO_ROOT/bench.py --model inception_v3_slim_old --steps 3 --warmup 3 > $GRAFT_REPO_ROOT/gpurun_out/r5/trace_inc2.log 2>&1 || { echo "trace failed"; exit 1; }
echo done
