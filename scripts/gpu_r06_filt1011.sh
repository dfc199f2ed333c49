#!/bin/bash
# Round 6: the LDS filter size on 2pc N=10 / 11 (8-byte entries: the compact filter needs B - L <= 30),
# SR_FILTER_LOG2 = 9 (default), 10, 8.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
bash scripts/gpu_env_ab.sh r06f1011/n10 2 "SR_X=0" "SR_FILTER_LOG2=10" "SR_FILTER_LOG2=8" -- --steps 5 --rm-count 10 || exit 1
bash scripts/gpu_env_ab.sh r06f1011/n11 1 "SR_X=0" "SR_FILTER_LOG2=10" "SR_FILTER_LOG2=8" -- --steps 2 --warmup 1 --rm-count 11 || exit 1
echo "filt1011 ok"
