#!/bin/bash
# Round 6: expand_route's grid cap (default two residencies) at about one residency (SR_ROUTE_GRID_MAX),
# config 4 (2pc N=11) on T = 8 / 4 virtual partitions: per-rank critical path.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
bash scripts/gpu_okey_sweep.sh 11 8 "SR_X=0" "SR_ROUTE_GRID_MAX=1536" "SR_ROUTE_GRID_MAX=1280" "SR_ROUTE_GRID_MAX=1792" || exit 1
bash scripts/gpu_okey_sweep.sh 11 4 "SR_X=0" "SR_ROUTE_GRID_MAX=1536" || exit 1
echo "route grid ok"
