#!/bin/bash
# Round 6: expand_fast's grid cap around one device residency (SR_GRID_MAX), 2pc N=9 / 10 / 11 and
# paxos C=6 (whose big levels stride).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
bash scripts/gpu_env_ab.sh r06grid2/n9 3 "SR_X=0" "SR_GRID_MAX=1536" "SR_GRID_MAX=1024" "SR_GRID_MAX=1280" "SR_GRID_MAX=1792" -- --steps 20 || exit 1
bash scripts/gpu_env_ab.sh r06grid2/n10 2 "SR_X=0" "SR_GRID_MAX=1536" -- --steps 5 --rm-count 10 || exit 1
bash scripts/gpu_env_ab.sh r06grid2/n11 1 "SR_X=0" "SR_GRID_MAX=1536" -- --steps 2 --warmup 1 --rm-count 11 || exit 1
bash scripts/gpu_env_ab.sh r06grid2/p6 2 "SR_X=0" "SR_GRID_MAX=1024" "SR_GRID_MAX=768" -- --steps 5 --model paxos --clients 6 || exit 1
echo "grid2 ok"
