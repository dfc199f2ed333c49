#!/bin/bash
# Round 6: parents per wave capped while the frontier grows (SR_PPW_ASC = 5 / 4 / off).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
bash scripts/gpu_env_ab.sh r06pa/n9 3 "SR_X=0" "SR_PPW_ASC=5" "SR_PPW_ASC=4" -- --steps 20 || exit 1
bash scripts/gpu_env_ab.sh r06pa/n10 2 "SR_X=0" "SR_PPW_ASC=5" "SR_PPW_ASC=4" -- --steps 5 --rm-count 10 || exit 1
bash scripts/gpu_env_ab.sh r06pa/n11 1 "SR_X=0" "SR_PPW_ASC=5" -- --steps 2 --warmup 1 --rm-count 11 || exit 1
bash scripts/gpu_env_ab.sh r06pa/il10 2 "SR_X=0" "SR_PPW_ASC=5" -- --steps 10 --model increment_lock --threads 10 || exit 1
echo "ppw asc ok"
