set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -m gpu > gpurun_out/t.log 2>&1 || { tail -30 gpurun_out/t.log; exit 1; }
tail -1 gpurun_out/t.log
for m in lenet vgg_16 inception_v3_slim_old; do
  timeout -k 10 300 python bench.py --model $m --steps 20 --warmup 5 > gpurun_out/all_$m.log 2>&1 || { echo "bench $m failed"; tail -20 gpurun_out/all_$m.log; exit 1; }
  grep -o '"value": [0-9.]*.\{0,120\}' gpurun_out/all_$m.log
done
TSTEPS=4 bash tools/gpu_runs/gpu_session.sh trainers > gpurun_out/trainers.log 2>&1 || { tail -30 gpurun_out/trainers.log; exit 1; }
grep -c "==" gpurun_out/trainers.log
