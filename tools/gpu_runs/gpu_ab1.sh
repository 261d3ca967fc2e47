set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_fused_gpu.py tests/test_fused_ops_gpu.py tests/test_engine.py > gpurun_out/fused_tests.log 2>&1 || { tail -30 gpurun_out/fused_tests.log; exit 1; }
tail -2 gpurun_out/fused_tests.log
VARIANTS="mat=;legacy=prologue:legacy;fused=prologue:fused" STEPS=6 ROUNDS=4 timeout -k 10 400 python -u tools/ab_step.py > gpurun_out/ab1.log 2>&1 || { tail -30 gpurun_out/ab1.log; exit 1; }
tail -8 gpurun_out/ab1.log
