#!/bin/bash
# GPU box session: tests, bench, kernel profile. Each GPU step has its own time limit; stop at first failure.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
MODE=${1:-all}
if [[ "$MODE" == *test* || "$MODE" == all ]]; then
  timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
  tail -3 gpurun_out/pytest_gpu.log
fi
if [[ "$MODE" == *bench* || "$MODE" == all ]]; then
  timeout -k 10 600 python bench.py --steps ${STEPS:-10} --warmup ${WARMUP:-3} ${BENCH_ARGS} > gpurun_out/bench.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/bench.log; exit 1; }
  tail -3 gpurun_out/bench.log
fi
if [[ "$MODE" == *prof* || "$MODE" == all ]]; then
  cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 2 ${BENCH_ARGS} > $GRAFT_REPO_ROOT/gpurun_out/prof.log 2>&1 || { echo "prof failed"; tail -30 $GRAFT_REPO_ROOT/gpurun_out/prof.log; exit 1; }
  cd $GRAFT_REPO_ROOT
  f=$(find gpurun_out/prof -name "*kernel_stats.csv" | head -1)
  echo "stats: $f"
  head -40 "$f" | cut -c1-220
fi
