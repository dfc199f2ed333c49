#!/bin/bash
# Round 6: parents per wave fixed for every level (SR_PPW_LOG2 = 3..6) against the per-level rule
# (engine.hpp ppw_for), 2pc N=9; the per-level kernel times of each line are compared afterwards.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
bash scripts/gpu_env_ab.sh r06ppw 2 "SR_X=0" "SR_PPW_LOG2=3" "SR_PPW_LOG2=4" "SR_PPW_LOG2=5" "SR_PPW_LOG2=6" -- --steps 20 || exit 1
echo "ppw ok"
