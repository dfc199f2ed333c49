#!/bin/bash
# Round 6: residencies per expand grid for wider states (default two): increment_lock N=11, paxos C=3 / C=6.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
bash scripts/gpu_env_ab.sh r06gr2/il11 1 "SR_X=0" "SR_GRID_RES=3" "SR_GRID_RES=4" -- --steps 2 --warmup 1 --model increment_lock --threads 11 || exit 1
bash scripts/gpu_env_ab.sh r06gr2/p3 2 "SR_X=0" "SR_GRID_RES=3" -- --steps 20 --model paxos --clients 3 || exit 1
bash scripts/gpu_env_ab.sh r06gr2/p6 2 "SR_X=0" "SR_GRID_RES=3" -- --steps 5 --model paxos --clients 6 || exit 1
echo "gridres2 ok"
