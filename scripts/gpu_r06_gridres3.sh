#!/bin/bash
# Round 6: residencies per expand grid for increment_lock (W = 2, every successor new).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
bash scripts/gpu_env_ab.sh r06gr3/il11 2 "SR_X=0" "SR_GRID_RES=4" "SR_GRID_RES=8" "SR_GRID_MAX=10000000" -- --steps 2 --warmup 1 --model increment_lock --threads 11 || exit 1
bash scripts/gpu_env_ab.sh r06gr3/il10 2 "SR_X=0" "SR_GRID_RES=4" "SR_GRID_RES=8" -- --steps 5 --warmup 1 --model increment_lock --threads 10 || exit 1
echo "gridres3 ok"
