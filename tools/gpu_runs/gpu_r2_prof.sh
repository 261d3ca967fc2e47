#!/bin/bash
# Round-2 evidence pass on one MI355X: full GPU test suite, ResNet-50 + Inception kernel-stat
# profiles, HBM bytes per ResNet-50 step, a 2-rank shared-GPU gloo rehearsal of bench.py phases.
set -o pipefail
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
rm -rf gpurun_out/prof gpurun_out/prof_inception_v3_slim_old gpurun_out/pmc_fetch gpurun_out/pmc_write
bash tools/gpu_runs/gpu_session.sh prof > gpurun_out/r2_prof_session.log 2>&1 || { tail -20 gpurun_out/r2_prof_session.log; exit 1; }
python3 tools/prof_summary.py $(find gpurun_out/prof -name "*kernel_stats.csv" | head -1) 5 30
MODELS=inception_v3_slim_old bash tools/gpu_runs/gpu_prof_models.sh || exit 1
bash tools/pmc_bw.sh > gpurun_out/pmc_session.log 2>&1 || { tail -20 gpurun_out/pmc_session.log; exit 1; }
cd $R
python3 tools/pmc_bw_report.py $(find gpurun_out/pmc_fetch -name "*counter_collection.csv" | head -1) $(find gpurun_out/pmc_write -name "*counter_collection.csv" | head -1) 3 30 > gpurun_out/r2_hbm_bytes.txt 2>&1 && tail -25 gpurun_out/r2_hbm_bytes.txt
timeout -k 10 300 python bench.py --gpus 2 --dist-backend gloo --model lenet --steps 5 --warmup 2 --graph 0 > gpurun_out/bench_gloo2_phases.log 2>&1 || { tail -20 gpurun_out/bench_gloo2_phases.log; exit 1; }
grep '"value"' gpurun_out/bench_gloo2_phases.log
