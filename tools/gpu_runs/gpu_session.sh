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
if [[ "$MODE" == *trainers* ]]; then
  # every entry script for a few steps on the GPU (synthetic data where the dataset is absent)
  for t in cifar10_cnn_bsp cifar10_alexnet_bsp cifar10_vgg_bsp cifar10_vgg_asp cifar10_resnet_bsp cifar10_cifarnet_bsp mnist_lenet_bsp imagenet_inception_bsp imagenet_inception_ssp; do
    timeout -k 10 300 python -m distributed_tensorflow_models_amd.trainers.$t --max_steps ${TSTEPS:-6} --synthetic_data --fresh --train_dir /tmp/tr_$t --data_dir /nonexistent > gpurun_out/trainer_$t.log 2>&1 || { echo "trainer $t failed"; tail -30 gpurun_out/trainer_$t.log; exit 1; }
    echo "== $t"; tail -n 2 gpurun_out/trainer_$t.log
  done
  timeout -k 10 300 python -m distributed_tensorflow_models_amd.trainers.cifar10_cnn_eval --checkpoint_dir /tmp/tr_cifar10_cnn_bsp --eval_dir /tmp/ev_cnn --run_once --data_dir /nonexistent > gpurun_out/eval_cnn.log 2>&1 || { echo "eval failed"; tail -30 gpurun_out/eval_cnn.log; exit 1; }
  tail -n 2 gpurun_out/eval_cnn.log
fi
