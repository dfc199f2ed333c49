#!/bin/bash
# Quick GPU pass for an expand_fast experiment: timing A/B of engine settings (per-level kernel
# times in each line's `levels.kernel_us`). Usage: scripts/gpu_quick_ab.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-q}
bash scripts/gpu_env_ab.sh $T/ppw9 1 "" "SR_PPW_LOG2=2" "SR_PPW_LOG2=3" "SR_PPW_LOG2=4" "SR_PPW_LOG2=5" "SR_PPW_LOG2=6" "SR_PPW_WAVES=16384" "SR_PPW_WAVES=65536" -- --steps 10 --warmup 3 || exit 1
bash scripts/gpu_env_ab.sh $T/ppw10 1 "" "SR_PPW_LOG2=4" "SR_PPW_LOG2=5" "SR_PPW_WAVES=16384" "SR_PPW_WAVES=65536" -- --steps 3 --warmup 1 --rm-count 10 || exit 1
