#!/bin/bash
# Round 5 session 13: Inception-v3 step kernel timelines, baseline .so vs the latency-shaped reductions.
set -o pipefail
mkdir -p gpurun_out/r5
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for v in base new; do
  if [ $v = base ]; then export DTM_KERNELS_SO=$R/ab_so/libdtm_kernels_base.so; else unset DTM_KERNELS_SO; fi
  rm -rf $R/gpurun_out/r5/prof_s13
  cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/r5/prof_s13 -o run --output-format csv -- python3 $R/bench.py --model inception_v3_slim_old --steps 4 --warmup 3 > $R/gpurun_out/r5/prof_s13.log 2>&1 || { echo "prof failed"; tail -20 $R/gpurun_out/r5/prof_s13.log; exit 1; }
  cd $R
  t=$(find gpurun_out/r5/prof_s13 -name "*kernel_trace.csv" | head -1); python3 tools/step_timeline.py "$t" > gpurun_out/r5/r5_s13_timeline_$v.txt; tail -1 gpurun_out/r5/r5_s13_timeline_$v.txt
done
rm -rf gpurun_out/r5/prof_s13
echo done
