#!/usr/bin/env bash
# Stop a launched run by its recorded PIDs (the reference ran `pkill python`, which also killed
# unrelated jobs).  bash scripts/clear.sh <model> <mode>   or   LOG_DIR=... bash scripts/clear.sh
here=$(cd "$(dirname "$0")/.." && pwd)
cd "$here"
exec python -m distributed_tensorflow_models_amd.parallel.launcher --stop --log_dir "${LOG_DIR:-$here/runs/${1}_${2:-bsp}}"
