#!/bin/bash
# Round 6: paxos launch knobs at the final sources: parents per wave fixed (SR_PPW_LOG2), LDS filter size
# (SR_FILTER_LOG2, default 10), C=3 and C=6.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
bash scripts/gpu_env_ab.sh r06pxk/p3 2 "SR_X=0" "SR_PPW_LOG2=3" "SR_PPW_LOG2=4" "SR_PPW_LOG2=5" "SR_FILTER_LOG2=9" "SR_FILTER_LOG2=11" -- --steps 20 --model paxos --clients 3 || exit 1
bash scripts/gpu_env_ab.sh r06pxk/p6 1 "SR_X=0" "SR_PPW_LOG2=4" "SR_PPW_LOG2=5" "SR_FILTER_LOG2=9" "SR_FILTER_LOG2=11" -- --steps 5 --model paxos --clients 6 || exit 1
echo "pxknobs ok"
