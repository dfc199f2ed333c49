#!/bin/bash
# Round 6: engine knobs at the new table (4-byte slots, 0.3 load), 2pc N=9: LDS filter size, chain
# depth, minimum waves per level.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
bash scripts/gpu_env_ab.sh r06k9 2 "SR_X=0" "SR_FILTER_LOG2=8" "SR_FILTER_LOG2=10" "SR_CHAIN_MAX=65536" "SR_PPW_WAVES=4096" "SR_PPW_WAVES=1024" -- --steps 20 || exit 1
echo "knobs9 ok"
