#!/usr/bin/env bash
# Single-node replacement for the reference train.sh: one rank per MI355X on this host.
#   bash scripts/train.sh <model> <bsp|asp|ssp> [trainer flags...]
# Env: NPROC (default: all visible GPUs), LOG_DIR (default runs/<model>_<mode>), EVAL=1 to start the
# evaluator 20 s later on the host (reference train.sh:57-59).
set -e
if [ -z "$1" ]; then
  echo "please specify model and sync mode (bsp, asp, ssp)!"
  exit 1
fi
model=$1; mode=${2:-bsp}; shift; [ $# -gt 0 ] && shift
here=$(cd "$(dirname "$0")/.." && pwd)
args=(--model "$model" --mode "$mode" --log_dir "${LOG_DIR:-$here/runs/${model}_${mode}}")
[ -n "$NPROC" ] && args+=(--nproc "$NPROC")
[ "${EVAL:-0}" = "1" ] && args+=(--eval)
cd "$here"
exec python -m distributed_tensorflow_models_amd.parallel.launcher "${args[@]}" -- "$@"
