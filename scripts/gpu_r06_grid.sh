#!/bin/bash
# Round 6: expand_fast's grid cap (default: two device residencies, blocks stride over further chunks)
# against other caps (SR_GRID_MAX), 2pc N=9 and N=10.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
bash scripts/gpu_env_ab.sh r06grid/n9 2 "SR_X=0" "SR_GRID_MAX=1536" "SR_GRID_MAX=4608" "SR_GRID_MAX=6144" "SR_GRID_MAX=1000000" -- --steps 20 || exit 1
bash scripts/gpu_env_ab.sh r06grid/n10 1 "SR_X=0" "SR_GRID_MAX=4608" "SR_GRID_MAX=1000000" -- --steps 5 --rm-count 10 || exit 1
echo "grid ok"
