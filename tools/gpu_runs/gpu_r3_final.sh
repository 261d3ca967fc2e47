#!/bin/bash
# Round-3 final evidence: GPU suite, smoke, benches (every BASELINE config), 8-rank gloo rehearsal of the driver's
# launch (ranks sharing the GPU), ResNet-50 kernel trace (per-kernel stats + two-stream step timeline).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3_final_pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -E "Error|assert|FAILED" gpurun_out/r3_final_pytest_gpu.log | head -20; tail -3 gpurun_out/r3_final_pytest_gpu.log; exit 1; }
tail -1 gpurun_out/r3_final_pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3_final_smoke.log 2>&1 || { tail -20 gpurun_out/r3_final_smoke.log; exit 1; }
tail -1 gpurun_out/r3_final_smoke.log
for m in resnet_v1_50 inception_v3_slim_old vgg_16 lenet; do
  timeout -k 10 300 python bench.py --model $m > gpurun_out/r3_final_bench_$m.log 2>&1 || { tail -20 gpurun_out/r3_final_bench_$m.log; exit 1; }
  tail -1 gpurun_out/r3_final_bench_$m.log
done
timeout -k 10 600 python bench.py --gpus 8 --dist-backend gloo --batch 32 --steps 3 --warmup 2 > gpurun_out/r3_final_gloo8.log 2>&1 || { tail -30 gpurun_out/r3_final_gloo8.log; exit 1; }
tail -1 gpurun_out/r3_final_gloo8.log
rm -rf gpurun_out/prof_final
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_final -o run -- python3 bench.py --steps 3 --warmup 2 > gpurun_out/r3_final_prof.log 2>&1 || { echo "prof failed"; tail -30 gpurun_out/r3_final_prof.log; exit 1; }
f=$(find gpurun_out/prof_final -name "*kernel_trace.csv" | head -1)
python3 tools/step_timeline.py "$f" > gpurun_out/r3_final_timeline_resnet.txt
tail -1 gpurun_out/r3_final_timeline_resnet.txt
s=$(find gpurun_out/prof_final -name "*kernel_stats.csv" | head -1)
cp "$s" gpurun_out/r3_final_resnet50_kernel_stats.csv
rm -rf gpurun_out/prof_final
