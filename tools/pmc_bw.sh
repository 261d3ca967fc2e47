# HBM traffic per kernel for a short ResNet-50 bench run: one rocprofv3 pass per counter group
# (FETCH_SIZE uses 3 TCC counters, WRITE_SIZE 2 - they cannot share a pass).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
ARGS=${BENCH_ARGS:-"--steps 2 --warmup 1"}
timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/pmc_fetch -o f -- python3 $R/bench.py $ARGS > $R/gpurun_out/pmc_fetch.log 2>&1 &&
timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/pmc_write -o w -- python3 $R/bench.py $ARGS > $R/gpurun_out/pmc_write.log 2>&1 &&
find $R/gpurun_out/pmc_fetch $R/gpurun_out/pmc_write -name "*.csv" | head -20
