set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_zoo_gpu.py tests/test_engine.py -m gpu > gpurun_out/t_fc.log 2>&1 || { tail -40 gpurun_out/t_fc.log; exit 1; }
tail -1 gpurun_out/t_fc.log
R=$GRAFT_REPO_ROOT
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_cnn -o run --output-format csv -- python3 -m distributed_tensorflow_models_amd.trainers.cifar10_cnn_bsp --max_steps 6 --synthetic_data --fresh --train_dir /tmp/tr_cnn --data_dir /nonexistent > $R/gpurun_out/prof_cnn.log 2>&1 || { tail -20 $R/gpurun_out/prof_cnn.log; exit 1; }
cd $R && f=$(find gpurun_out/prof_cnn -name "*kernel_stats.csv" | head -1) && cut -c1-150 "$f" | head -30
