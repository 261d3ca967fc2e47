set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_fused_ops_gpu.py tests/test_fused_gpu.py tests/test_kernels_gpu.py -m gpu > gpurun_out/t_bnout.log 2>&1 || { tail -30 gpurun_out/t_bnout.log; exit 1; }
tail -1 gpurun_out/t_bnout.log
VARIANTS="${VARIANTS:-fuse=;nofuse=bnout:0;nosact=sact:0}" ROUNDS=5 timeout -k 10 400 python -u tools/ab_step.py > gpurun_out/ab_bnout.log 2>&1 || { tail -20 gpurun_out/ab_bnout.log; exit 1; }
tail -3 gpurun_out/ab_bnout.log
