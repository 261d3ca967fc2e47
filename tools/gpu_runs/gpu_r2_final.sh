#!/bin/bash
# Round-2 final evidence: GPU suite, smoke, every bench config, 2-rank shared-GPU bench rehearsal, ResNet-50 profile.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_final.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_gpu_final.log; exit 1; }
tail -2 gpurun_out/pytest_gpu_final.log
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
bash tools/gpu_runs/gpu_bench_all.sh > gpurun_out/bench_all_final.log 2>&1 || { tail -20 gpurun_out/bench_all_final.log; exit 1; }
cat gpurun_out/bench_all_final.log
timeout -k 10 300 python bench.py --gpus 2 --dist-backend gloo --steps 5 --warmup 2 > gpurun_out/bench_gloo2_final.log 2>&1 || { tail -20 gpurun_out/bench_gloo2_final.log; exit 1; }
grep '"value"' gpurun_out/bench_gloo2_final.log | cut -c1-400
rm -rf gpurun_out/prof
bash tools/gpu_runs/gpu_session.sh prof > gpurun_out/prof_session_final.log 2>&1 || { tail -20 gpurun_out/prof_session_final.log; exit 1; }
rm -rf gpurun_out/prof_inception_v3_slim_old gpurun_out/prof_vgg_16
MODELS="inception_v3_slim_old vgg_16" bash tools/gpu_runs/gpu_prof_models.sh > gpurun_out/prof_models_final.log 2>&1 || { tail -20 gpurun_out/prof_models_final.log; exit 1; }
python3 tools/prof_summary.py $(find gpurun_out/prof -name "*kernel_stats.csv" | head -1) 5 12
